// decoder.hpp — host/device shared definitions of the gfx950 LDPC decoder.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qldpc {

// Per-slot metadata word (slot-major [slot][lane], one uint32 per CSR edge).
constexpr uint32_t META_COL_MASK = 0xFFFFFu;   // bit id (n <= 2^20)
constexpr int META_KPOS_SHIFT = 20;            // position of the edge in its bit's check list
constexpr uint32_t META_KPOS_MASK = 0x1FFu;    // dv < 511 (511 marks a V2 dummy slot)
constexpr uint32_t META_START = 1u << 29;      // first edge of its row
constexpr uint32_t META_END = 1u << 30;        // last edge of its row
constexpr uint32_t META_VALID = 1u << 31;      // slot holds an edge (tail padding otherwise)
constexpr int MAX_DV = (int)META_KPOS_MASK;
constexpr int MAX_N = 1 << 20;

// Registers available for per-edge messages in the register-resident variant.
constexpr int EPL_REG = 40;
// Lane stride of the register variant's metadata groups (== max lanes).
constexpr int REG_TSTRIDE = 1024;

enum Variant : int {
    VAR_REG_LDS = 0,  // messages in VGPRs, totals/rows in LDS       (n <~ 14k)
    VAR_GLB_LDS = 1,  // messages in per-workgroup global scratch, totals/rows in LDS
    VAR_GLB_GLB = 2,  // everything per-frame in global scratch     (n = 100k)
    VAR_V2 = 3,       // wave-aligned register kernel (decoder_v2.hip)
};

// Register slots per lane of the V2 instantiations.  (A third, 84 slots x 8
// waves, holds no more edges than 56 x 12 and its SPA build falls back to a
// scratch array, so it is not built.)
constexpr int V2_R_TIGHT = 40, V2_R_SMALL = 44, V2_R_MID = 56;
#ifndef QL_SPLIT_R
#define QL_SPLIT_R 40  // split frames' slots per lane (A/B: 44, 48 with a matching capi build)
#endif
constexpr int V2_R_SPLIT = QL_SPLIT_R;
// Split frames may add this many message slots per lane in per-workgroup
// global scratch to the V2_R_SPLIT register/LDS slots (round 6): more edges
// per part, so fewer parts per frame and more frames per XCD.  The planner
// takes them only when they raise frames per XCD by >= 4/3 (capi.hip
// plan_v2_split).
#ifndef QL_SPLIT_RG
#define QL_SPLIT_RG 12
#endif
constexpr int V2_RG_SPLIT = QL_SPLIT_RG;
static_assert(V2_RG_SPLIT > 0 && V2_RG_SPLIT % 4 == 0 && V2_R_SPLIT + V2_RG_SPLIT <= 64,
              "split scratch slots: groups of four, <= 64 slots in all");
constexpr int V2_CODES_CAP = 20480;  // V2: bits per frame whose palette indices fit LDS (n <= this)
// Hybrid instantiation: 44 VGPR slots + this many slots in per-workgroup global scratch.
constexpr int V2_RG_HYBRID = 20;
// SPA-family register kernels at V2_R_TIGHT keep this many message slots in LDS
// (when the frame's LDS image leaves room) instead of VGPRs.  5: the C2 image
// is then 159.8 KiB, and the kernel spills fewer VGPRs to scratch than with 4
// (same-box A/B: 0.6% faster decode, profiles/r04/ab_rl5.txt).
#ifndef QL_RL
#define QL_RL 5
#endif
constexpr int V2_RL = QL_RL;
// Workgroup size each V2 instantiation is compiled for (its VGPR budget).
constexpr __host__ __device__ int v2_threads_for(int R) { return R <= V2_R_SMALL ? 1024 : 768; }

// Phase ids of the diagnostic stamp build (QL_PHASE_STAMPS).
enum StampId : int {
    ST_SETUP, ST_SETUP_WAIT, ST_S, ST_S_WAIT, ST_CN1, ST_CN1_WAIT, ST_CN2, ST_CN2_WAIT, ST_CN3,
    ST_VN0, ST_VN0_WAIT, ST_VNK, ST_VNK_WAIT, ST_OUT, ST_OUT_WAIT, NUM_STAMPS
};
static const char *const STAMP_NAMES[NUM_STAMPS] = {
    "setup", "setup_wait", "synd", "synd_wait", "cn1", "cn1_wait", "cn2", "cn2_wait", "cn3",
    "vn_init", "vn_init_wait", "vn_phases", "vn_phases_wait", "out", "out_wait"};

struct DecodeArgs {
    // graph (device pointers; shared by every frame)
    int n, m, E, T, EPL, dv_max, max_dc;
    const uint32_t *slot_meta;  // [ceil(EPL/4)][T][4]: uint4 per 4 slots
    const int32_t *lane_row0;   // [T] row of slot 0 (or -1)
    const int32_t *lane_head;   // [T] leading slots that finish a row begun in lane-1
    const int32_t *lane_nst;    // [T] V2: rows started in the lane
    const int32_t *lane_epl;    // [T] V2: slots of the lane's wave (uniform per wave)
    const int32_t *ell_col;     // [max_dc][m] bit ids of each row, row-ELL, slot-major
    const int32_t *row_deg;     // [m]
    // decoder parameters
    int alg, max_it, thr_on;
    double thr, primary, secondary;
    // SPA edge-form constants, computed by the host C library (capi.hip):
    double spa_tlim;  // tanh(min(thr, 44) / 2.)  (1 when clipping is off)
    double spa_ctop;  // 2. * atanh(1 - 2^-53)
    // frames
    int batch;
    const double *llr;      // [batch][n]
    const uint8_t *synd;    // [batch][m]
    uint8_t *bits;          // [batch][n]
    uint32_t *iters;        // [batch]
    uint8_t *ok;            // [batch]
    double *post;           // [batch][n] or nullptr
    // scheduling / scratch
    int *frame_counter;
    const int32_t *frame_order;   // [batch] claim order (order.hip); nullptr: index order
    double *scratch;              // per-workgroup scratch (variants 1, 2)
    long long scratch_wg_doubles; // doubles per workgroup
    uint64_t *stamps;             // diagnostic build only: [wg][wave][NUM_STAMPS]
    // V2 frame format: channel LLRs as a 4-entry palette + 2-bit codes
    int nc;                  // code bytes per frame = ceil(n / 4)
    const uint8_t *codes;    // [batch][nc]
    const double *palette;   // [batch][4]
    const uint8_t *pal_ok;   // [batch]; 0 -> the decoder gathers llr[] instead
    int n_iso;               // bits with no check (dv = 0): total = llr
    const int32_t *iso_bits; // [n_iso]
    int v2R;                 // register slots of the V2 instantiation to launch
    int v2RG;                // + slots in per-workgroup global scratch (0 or V2_RG_HYBRID)
    const uint64_t *vn_mask; // [waves][dv_max]: slots holding a kk-th bit edge, per wave
    const uint64_t *vn_exec; // [waves][dv_max][slots]: lanes whose slot holds a kk-th bit edge
    // V2 hybrid: VN terms k >= vn_k0 are staged in scratch by the message pass
    // and summed per bit in one gather pass (bits sorted by degree, descending).
    int vn_k0;                      // first staged term (dv_max: none)
    int n_hd;                       // bits with degree > vn_k0
    const int32_t *hd_bits;         // [n_hd]
    const int32_t *hd_dv;           // [n_hd]
    int hd_uniform_dv;              // > 0: hd_bits[i] == i and hd_dv[i] == this for every i
    const int32_t *stage_off;       // [dv_max]: offset of term kk's block in the stage
    const uint32_t *slot_meta2;     // like slot_meta: stage index of the slot's edge
    long long stage_wg_offset;      // doubles from a workgroup's scratch base to its stage
    const int32_t *row_orig;        // V2: layout row -> original row (syndrome index)
    // V2 scan (one workgroup per frame, register slots only): the row
    // structure as lane masks and per-lane row slot masks (capi.hip)
    const uint64_t *row_sem;        // [waves][slots][4]: the lanes whose slot starts / ends a row / parks a tail
    const uint64_t *row_rmask;      // [nst_max][T]: slots of the lane's j-th started row; bit 63: open
    int nst_max;
    // V2 split frames (split_k > 1 workgroups of one XCD per frame)
    int split_k;                    // parts per frame (1: not split)
    int split_mrows;                // rows of the largest part (LDS rows array)
    int split_slots;                // group slots per XCD in the arrays below
    const int32_t *part_row0;       // [split_k + 1] first layout row of each part
    int *split_claim;               // [16] per-XCD claim counters
    int *split_pub;                 // [16][slots] frame + 1, published by rank 0
    int *split_sync;                // [16][slots] group barrier arrivals
    int *split_mis;                 // [16][slots] iteration + 1 of the last row mismatch
    double *gtotal;                 // [batch][n + 1] the frames' totals
    int *split_err;                 // set when a part group failed to meet (results void)
    double *gstage;                 // [batch][stage_frame_doubles] split frames' VN stage
    long long stage_frame_doubles;
    // Split-frame exchange layout (nullptr xoff: the term-major stage).  Part p
    // owns bits [n p / K, n (p + 1) / K) in split_nc chunks of split_cb; the
    // stage is one region per (owner part, chunk, kpos), each holding its terms
    // in (writer wave, slot, lane) order, so a writing wave fills whole lines
    // and the owner reads each region front to back, adding every term into
    // an LDS sum at the bit's chunk-local index xbit[position].
    int split_cb, split_nc;
    const int32_t *xoff;            // [K * nc * dv_max + 1] region starts (doubles into the frame's stage)
    const uint16_t *xbit;           // [stage_frame_doubles] chunk-local bit of each stage position
    // v1 global-slot kernels, unsorted adjacency (occurrence pairing): input
    // slot s of the next check-node pass gets total[pair_col[s]] -
    // c2b[pair_src[s]] (both [k][lane]); the values go through a slot-major
    // buffer at pair_buf_off doubles into the workgroup's scratch.  nullptr: off.
    const int32_t *pair_src;
    const int32_t *pair_col;
    long long pair_buf_off;
    // V2 min-sum bit gather (VNG, dv_max <= 4): the message pass records per
    // edge two bits (b2c <= 0, |b2c| == min1) in LDS, and one pass per bit
    // rebuilds its messages from its rows' aggregates and sums them in order.
    const uint2 *vn_rows;           // [n]: four u16 layout rows per bit, kpos order (0xFFFF: none); null: off
    // Hybrid shape (irregular codes): a bit's edges are padded to chunks of
    // four; vn_rows then holds the rows per chunk ([chunks], padding: row 0),
    // slot_meta2 each slot's padded edge position, and the gather walks bits
    // in degree order: vng_bits[i] = {bit, first chunk | dv << 24}.
    const uint2 *vng_bits;
    // Min-sum: the factor/offset can push |message| above its selected
    // minimum (|NMSA factor| > 1, negative offset, or NaN): clip every message.
    int ms_clip_later;
    // Hybrid min-sum whose row aggregates do not fit LDS beside the totals
    // (C5 R=0.5: m = 5120): rowAB lives in the workgroup's global scratch
    // (L2-resident) at this offset in doubles; -1: rows in LDS.
    long long rows_wg_offset;
    int rows_lds;                   // ... of which the leading rows_lds layout rows stay in LDS (m: all)
    int rows_lds_waves;             // = the rows of waves 0 .. rows_lds_waves - 1
    const int32_t *wave_rows;       // V2: first layout row of each wave (+ m)
    int rows_copy;                  // ... the others' message pass reads an LDS copy of its rows
    // Bank-aware bit labels (relabel.cpp; one-workgroup register shapes): the
    // graph's metadata and the frame codes use labels, llr / bits / posterior
    // the reference's bit ids.  nullptr: identity.
    const int32_t *col_orig;        // [n] label -> bit id (the frame codes the kernel reads are in labels)
    const int32_t *col_lab;         // [n] bit id -> label (outputs: bits / posterior in bit ids)
    // ... a frame the palette cannot hold is copied into label order at frame
    // setup, into its workgroup's scratch at this offset (doubles); -1: none
    long long llr_lab_wg_offset;
    // Per-frame decode span (nullable): [batch][2] s_memrealtime ticks (100 MHz)
    // at the frame's claim and at its results — the trial's own time inside the
    // batch (the reference times each trial's QKD_LDPC call, src/simulation.cpp:559-568)
    uint64_t *frame_clk;
};

// Frequency of s_memrealtime (gfx9: a constant 100 MHz clock).
constexpr double FRAME_CLK_HZ = 100.0e6;

// The persistent decoders' frame claim: the next frame of the launch's claim
// order (order.hip; results never depend on it).  >= batch: none left.
__device__ __forceinline__ int claim_frame(const DecodeArgs &a) {
    const int c = atomicAdd(a.frame_counter, 1);
    return (a.frame_order && c < a.batch) ? a.frame_order[c] : c;
}

// Dynamic LDS bytes / scratch doubles a variant needs for this shape.
size_t lds_bytes_for(int variant, int n, int m, int T);
long long scratch_doubles_for(int variant, int n, int m, int T, int EPL);

// Launch the persistent decoder: grid = `workgroups`, block = args.T.
hipError_t launch_decode(int variant, const DecodeArgs &a, int workgroups, size_t lds_bytes,
                         hipStream_t stream);
// Max resident workgroups per CU for (variant, alg, T, lds).
hipError_t occupancy(int variant, int alg, int T, size_t lds_bytes, int *blocks_per_cu);

// The environment variable `name` under the diagnostic switch QLDPC_DIAG=1, else NULL (capi.hip):
// the only way the library reads its QLDPC_* A/B knobs.
const char *qldpc_diag_env(const char *name);
constexpr size_t LDS_MAX_BYTES = 160 * 1024;
// Opt kernel k in to `bytes` of dynamic LDS (hipFuncAttributeMaxDynamicSharedMemorySize)
// on the current device.  The limit per (device, kernel) only ever rises,
// under one process-wide mutex: a
// per-launch value set by one thread could otherwise lower the limit between
// another thread's set and its launch (decoder.hip).
hipError_t allow_dynamic_lds(const void *k, size_t bytes);
// Dynamic LDS of the frame builders: the keys (+ punctured draws, the extended
// key) as bit words.  Beyond LDS_MAX_BYTES (plain frames: n > 655,360; rate-
// adapted: n > ~436k) the entries refuse the graph with QLDPC_EUNSUP.
inline size_t build_frames_lds(int n) { return 2 * (size_t)((n + 31) / 32) * sizeof(uint32_t); }
inline size_t build_frames_ra_lds(int n, int n_punct) {
    return (2 * (size_t)((n + 31) / 32) + (size_t)((n_punct + 31) / 32) + 2 * (size_t)((n + 63) / 64)) *
           sizeof(uint32_t);
}
// Threads per frame of the one-workgroup-per-frame byte kernels (frame build,
// claim weight, key compare): 256, or 1024 for frames of >= 32768 bits, whose
// batches (C4: 128 frames) leave most CUs idle at 4 waves per frame.
inline int aux_frame_threads(int n) { return n >= 32768 ? 1024 : 256; }
hipError_t launch_build_frames(int n, int m, int max_dc, const int32_t *ell_col, const int32_t *row_deg,
                               int batch, const uint8_t *alice, const uint8_t *bob, const double *log_p,
                               double *llr, uint8_t *synd, uint8_t *codes, double *palette, uint8_t *pal_ok,
                               const int32_t *col_orig, hipStream_t stream);

// LDS bytes of a V2 launch; R/RG select the shape (whether message slots live in LDS).
// rows_lds: min-sum row aggregates kept in LDS on the hybrid shape (-1: all m).
size_t lds_bytes_v2(int alg, int n, int m, int T, bool split = false, int R = 0, int RG = 0, int rows_lds = -1,
                    int gcb = 0);
// Whether a V2 shape can run the min-sum bit gather (DecodeArgs::vn_rows):
// the dv <= 4 register shape, or the hybrid shape when the padded edge
// positions' two code bits fit the LDS byte area.
bool v2_vng_ok(int alg, int R, int RG, int split_k, int dv_max, int m);
// Split frames: whether the SPA layout keeps its LDS message slots at gcb exchange-gather bits.
bool v2_split_rl_fits(int n, int mrows, int gcb, int pl);
constexpr int V2_VNG_DUMMY_CHUNKS = 64;  // hybrid: one scratch code byte per lane for dummy slots
hipError_t launch_decode_v2(const DecodeArgs &a, int workgroups, size_t lds_bytes, hipStream_t stream);
hipError_t occupancy_v2(int R, int RG, int split_k, int alg, int T, size_t lds_bytes, int *blocks_per_cu);
hipError_t launch_palettize(int n, int nc, int batch, const double *llr, uint8_t *codes, double *palette,
                            uint8_t *pal_ok, const int32_t *col_orig, hipStream_t stream);
// Trial generator workspace (uint32 words) of `batch` trials.
size_t trials_scratch_words(int n, uint64_t n_err, int n_punct, int batch);
// The Xoshiro256 state after `draws` draws from a Xoshiro-cpp-seeded generator,
// by the jump matrix the trial generator's second wave uses (host; a check).
int xoshiro_jump_check(uint64_t seed, uint64_t draws, uint64_t *state_out);
hipError_t launch_trials(int n, uint64_t n_err, int batch, const uint64_t *seeds, uint64_t seed_add, uint8_t *alice,
                         uint8_t *bob, uint32_t *scratch, int n_punct, uint8_t *punct_alice, uint8_t *punct_bob,
                         hipStream_t stream);
hipError_t launch_build_frames_ra(int n, int m, const int32_t *ell_col, const int32_t *row_deg, const uint8_t *cls,
                                  const int32_t *src, int n_punct, int batch, const uint8_t *alice, const uint8_t *bob,
                                  const uint8_t *palice, const uint8_t *pbob, const double *log_p, uint8_t *alice_ext,
                                  double *llr, uint8_t *synd, uint8_t *codes, double *palette, uint8_t *pal_ok,
                                  const int32_t *col_orig, hipStream_t stream);
// Claim order of a batch: frames by ascending weight of the channel decision's
// syndrome mismatch (order.hip).  llr is read only for frames without codes.
size_t frame_weight_lds(int n);
hipError_t launch_frame_order(int n, int m, const int32_t *ell_col, const int32_t *row_deg, int batch,
                              const uint8_t *synd, const double *llr, const uint8_t *codes,
                              const double *palette, const uint8_t *pal_ok, int32_t *weight, int32_t *order,
                              const int32_t *col_orig, hipStream_t stream);
hipError_t launch_math_selftest(int fn, int count, const double *in, double *out, hipStream_t stream);
hipError_t launch_keys_match(int batch, int n, const uint8_t *alice, const uint8_t *bits,
                             uint8_t *match, hipStream_t stream);

}  // namespace qldpc
