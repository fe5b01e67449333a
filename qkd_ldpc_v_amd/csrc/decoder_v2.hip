// decoder_v2.hip — wave-aligned register decoder (variant V2) for gfx950.
//
// Same decoders and bit-exactness contract as decoder.hip (reference
// src/qkd_ldpc_algorithm.cpp:3-1029), restructured to cut barriers:
//   * rows are dealt to WAVES (contiguous blocks, balanced by edges), then a
//     wave's edges to its 64 lanes, EPL per lane (<= R, compile-time register
//     slots).  A row may straddle two lanes of one wave, never two waves, so a
//     split row's running product / min-sum aggregate / parity moves by one
//     wave shuffle instead of an LDS round trip and two barriers;
//   * the syndrome check (reference :86,101-107 and :745-776) is fused into the
//     check-node pass, which gathers every total[col] anyway: each row's
//     parity of the current hard decision is folded into the row scan;
//   * VN phase 0 (total = llr + first message) is fused into the message
//     pass; the channel LLRs live in LDS as a 4-entry palette + 2-bit codes
//     (every frame the reference builds has <= 4 distinct LLRs: +-log_p, 1e-4,
//     DBL_MAX); frames that do not fit gather llr[] from global instead.
// Per iteration: 1 barrier after the check-node scan, 1 after the message
// pass, 1 per remaining VN phase (dv_max - 1).
#include <type_traits>

#include "decoder_common.hpp"

namespace qldpc {

namespace {

using namespace dev;

constexpr int V2_CTRL = 16;  // s_frame, mismatch epoch
#ifndef QL_VN_BATCH
#define QL_VN_BATCH 2
#endif
constexpr int V2_VN_BATCH = QL_VN_BATCH;  // VN phases: slot groups per LDS round trip
#ifndef QL_SPLIT_DEFER
// split frames: the exit test after the message pass, a workgroup barrier
// between scan and message pass (1); 0: the test first (A/B builds only; the
// round-5 wave-local-fence arm measured equal and was removed)
#define QL_SPLIT_DEFER 1
#endif
static_assert(QL_SPLIT_DEFER == 0 || QL_SPLIT_DEFER == 1, "QL_SPLIT_DEFER: 0 or 1");
#ifndef QL_MSG_PF
#define QL_MSG_PF 1  // stage-writing message passes request the next group's metadata early
#endif
#ifndef QL_XG_UNROLL
#define QL_XG_UNROLL 4  // split exchange gather: terms per thread per load round (8: spills, 10% slower C4)
#endif
#ifndef QL_GH_PF
#define QL_GH_PF 1  // hybrid bit gather: the next bit's entry requested one bit ahead
#endif
#ifndef QL_SPLIT_TANH_W
#define QL_SPLIT_TANH_W 1  // split-frame SPA: tanh's expm1 table in the word form (exact_math.h Expm1Bw)
#endif
#ifndef QL_HOIST_LLR
#define QL_HOIST_LLR 0  // (A/B) SPA message pass: the kpos-0 channel LLR requested first
#endif
#ifdef QL_NO_ROWSCAN
constexpr bool V2_ROWSCAN_ON = false;  // A/B only: SPA scan with per-slot flag bookkeeping
#else
constexpr bool V2_ROWSCAN_ON = true;
#endif

__host__ __device__ inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// LDS of one frame.  total has n + 1 entries: total[n] is the column of the
// dummy slots that pad every lane of a wave to the same slot count.
// The palette, the per-bit palette indices and the totals sit at fixed
// offsets, so their LDS addresses are instruction immediates (no base
// register): codes hold up to V2_CODES_CAP bits (plan_v2 enforces n <= it).
constexpr int V2_PAL_OFF = V2_CTRL;                    // 4 doubles
constexpr int V2_CODES_OFF = V2_PAL_OFF + 32;          // one palette index byte per bit
constexpr int V2_TOTAL_OFF = V2_CODES_OFF + V2_CODES_CAP;
static_assert(V2_TOTAL_OFF % 16 == 0 && V2_TOTAL_OFF < 65536, "ds offset immediates are 16-bit");
// SPA iteration 0 on frames whose channel LLRs are all +-L: entry 0 is
// t0 = tanh(L / 2.), entry d >= 1 the clipped 2 * atanh(|rp| / t0) of a row of
// degree d (rows have <= 32 edges: plan_v2).
constexpr int V2_A0_ENTRIES = 64;
// Split frames (several workgroups per frame): the totals live in global
// memory and the palette indices are read from the 2-bit global codes; LDS
// holds the palette and this part's rows (m = the largest part's row count).
struct V2Layout {
    size_t total, rows, rowflag, tail, tailneg, a0tab, ctab, msl, codes, palette, syn, bytes;
    // ls: the lane stride of the LDS message slots (the workgroup's lanes;
    // split parts of 8 waves use 512)
    __host__ __device__ V2Layout(int n, int m, int, int T, bool minsum, bool split = false, int rl = 0,
                                 bool rowscan = false, int gcb = 0, int ls = REG_TSTRIDE) {
        palette = V2_PAL_OFF;
        codes = split ? 0 : V2_CODES_OFF;
        size_t o = split ? V2_CODES_OFF : V2_TOTAL_OFF;
        total = o; o = split ? o : al16(o + (size_t)(n + 1) * 8);
        rows = o; o = al16(o + (size_t)m * (minsum ? 16 : 8));  // SPA: product; min-sum: {min1, min2}
        rowflag = o;  // (min-sum row flags ride in the sign bits of rowAB: none here)
        tail = o;     // (min-sum: a lane's tail aggregate is parked in its row's rowAB entry)
        tailneg = o;
        a0tab = o; o = al16(o + (minsum ? 0 : (size_t)V2_A0_ENTRIES * 8));  // SPA: iteration-0 table
        // split frames' exchange gather: gcb bit sums in LDS over the rows and
        // the iteration-0 table, both dead between the message pass and the scan
        if (split && gcb > 0 && al16(rows + (size_t)gcb * 8) > o) o = al16(rows + (size_t)gcb * 8);
        ctab = o; o = al16(o + (minsum ? 0 : (size_t)ql_exact::EXPM1_CLASSES * (sizeof(ql_exact::Expm1A) + sizeof(ql_exact::Expm1B))));  // SPA: tanh's expm1 classes
        msl = o; o = al16(o + (size_t)rl * ls * 8);  // message slots held in LDS
        // one workgroup per frame: the rows' target syndrome bits as sign words
        // (s << 31), in the palette-index area past the codes when it has room
        syn = 0;
        if (rowscan && !split) {
            // (a spare word past the per-bit bytes: the min-sum bit gather's
            // dummy slots OR their record bits into it)
            const size_t cs = V2_CODES_OFF + al16((size_t)n + 4);
            if (cs + (size_t)m * 4 <= (size_t)V2_CODES_OFF + V2_CODES_CAP) {
                syn = cs;
            } else {
                syn = o;
                o = al16(o + (size_t)m * 4);
            }
        }
        bytes = o;
    }
};

template <int R>
constexpr int v2_max_threads() { return v2_threads_for(R); }

// R message slots per lane in VGPRs plus RG in global scratch; S = R + RG
// slots in all.  Slots that can belong to a lane's tail (the end of a row
// begun in the lane before): the planner keeps max_dc <= 32, so head <= 31.
template <int S>
constexpr int v2_tail_slots() { return S < 32 ? S : 32; }

// SPLIT: a frame is decoded by a.split_k workgroups of one XCD (planner
// parts: contiguous blocks of 16 waves' rows), which meet at every phase
// boundary through a global arrival counter; totals are in global memory.
// One 16-byte row aggregate {min1, min2} through a buffer resource.
__device__ __forceinline__ double2 ld_row16(__amdgpu_buffer_rsrc_t rs, int r) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, r * 16, 0, 0);
    double2 d;
    d.x = __builtin_bit_cast(double, ((unsigned long long)v.y << 32) | v.x);
    d.y = __builtin_bit_cast(double, ((unsigned long long)v.w << 32) | v.z);
    return d;
}
__device__ __forceinline__ void st_row16(__amdgpu_buffer_rsrc_t rs, int r, double2 d) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const unsigned long long x = __builtin_bit_cast(unsigned long long, d.x);
    const unsigned long long y = __builtin_bit_cast(unsigned long long, d.y);
    u32x4 v;
    v.x = (unsigned int)x;
    v.y = (unsigned int)(x >> 32);
    v.z = (unsigned int)y;
    v.w = (unsigned int)(y >> 32);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, r * 16, 0, 0);
}

template <bool SPLIT, int RL, bool RGLB, bool ROWSCAN, int R, int PL>
__device__ __forceinline__ V2Layout v2_layout(const DecodeArgs &a, bool minsum) {
    if constexpr (SPLIT)
        return V2Layout(a.n, a.split_mrows, a.nc, a.T, minsum, true, RL, false, a.split_cb, PL);
    else return V2Layout(a.n, RGLB ? a.rows_lds : a.m, a.nc, a.T, minsum, false, RL, ROWSCAN);
}

// Whether a launch runs the LDS-slot instantiation (RL = V2_RL): SPA family,
// register shape V2_R_TIGHT, and the frame's LDS image plus the slots fit.
__host__ __device__ inline bool v2_use_rl(int alg, int R, int RG, bool split, int n, int m, int T) {
    if (alg > 1 || R != V2_R_TIGHT || RG != 0 || split || T > REG_TSTRIDE) return false;
    return V2Layout(n, m, (n + 3) / 4, T, false, false, V2_RL, V2_ROWSCAN_ON).bytes <= 160 * 1024;
}
// Split frames keep their totals in global memory, so a part's LDS holds only
// its rows: the SPA family keeps v2_rl_split(pl) of the 40 message slots there
// (the register kernel otherwise spills in its slot loops) — 12 in 8-wave
// parts (80 KiB of LDS each), 16 in 16-wave parts (160 KiB; round 6, C4 (ii)'s
// 16-wave scratch-slot plan: decode −1.6 % against 12, profiles/r06/rl_split/;
// 16 in 8-wave parts was 3–6 % slower on the stand-in).  m: the largest
// part's row count.
#ifndef QL_RL_SPLIT
#define QL_RL_SPLIT 12
#endif
#ifndef QL_RL_SPLIT_16
#define QL_RL_SPLIT_16 16
#endif
constexpr int V2_RL_SPLIT = QL_RL_SPLIT;
constexpr int V2_RL_SPLIT_16 = QL_RL_SPLIT_16;
// pl: the part's lanes (1024, or 512 for parts of 8 waves, two per CU: half
// the LDS each).
__host__ __device__ constexpr int v2_rl_split(int pl) { return pl == REG_TSTRIDE ? V2_RL_SPLIT_16 : V2_RL_SPLIT; }
__host__ __device__ inline bool v2_use_rl_split(int alg, int n, int mrows, int gcb, int pl = REG_TSTRIDE) {
    return alg <= 1 && V2Layout(n, mrows, (n + 3) / 4, pl, false, true, v2_rl_split(pl), false, gcb, pl).bytes <=
                           (size_t)160 * 1024 * pl / REG_TSTRIDE;
}

constexpr int V2_SPLIT_SPIN_LIMIT = 1 << 22;  // ~seconds of polling: a broken group ends, never hangs

// Barrier of a split frame's part group: every wave's global stores reach L2
// (the group shares this XCD's L2), one arrival per workgroup, a bounded wait
// for the group's count, then the frame's totals are re-read past L1.
__device__ __forceinline__ void group_sync(int *ctr, int target, int *err) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (++spins >= V2_SPLIT_SPIN_LIMIT) {  // reported; the frame's results are void
                atomicOr(err, 1);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    asm volatile("buffer_inv sc1" ::: "memory");
}

// VNG (min-sum family, dv_max <= 4, not split): no VN phases.  The message
// pass ORs two bits per edge into a per-bit byte in LDS (the palette-index
// area: the channel LLR is then read from the frame's 2-bit global codes);
// after one barrier each thread rebuilds a bit's messages from its rows'
// aggregates — the same operations the message pass ran — and sums them in
// kpos order onto the channel LLR (std::accumulate order, :78).
// RGLB (hybrid min-sum bit gather only): the row aggregates live in the
// workgroup's global scratch instead of LDS (a.rows_wg_offset).
// LDS byte offset of total[col] for a slot's metadata word, col * 8, in one
// v_mad_u32_u16 instead of a mask and a shift-add: whenever the totals live in
// LDS the bit ids (dummy column n included) are below 2^16 — (n + 1) * 8
// bytes fit 160 KiB, and launch_decode_v2 checks n < 2^16 — so the low 16
// bits of the word are the bit id and its kpos / flag bits are ignored.
// (base: the LDS address of total[0], the mad's addend)
typedef __attribute__((address_space(3))) double lds_f64;
__device__ __forceinline__ lds_f64 *col_off8(uint32_t mt, uint32_t base) {
    uint32_t o;
    asm("v_mad_u32_u16 %0, %1, 8, %2" : "=v"(o) : "v"(mt), "s"(base));
    return (lds_f64 *)(uintptr_t)o;
}

// PL (split frames): the part's lanes — 1024 (16 waves, one part per CU) or
// 512 (8 waves, two parts per CU; the register budget stays that of 1024
// threads).  The graph's per-part arrays keep a stride of REG_TSTRIDE lanes /
// 16 waves either way (planner: parts of 8 waves leave waves 8..15 empty).
template <int ALG, int R, int RG, bool SPLIT, int RL = 0, bool VNG = false, bool RGLB = false, int PL = REG_TSTRIDE>
__global__ void __launch_bounds__(v2_max_threads<R>()) decode_v2_kernel(DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool SPA_FAM = (ALG == 0 || ALG == 1);
    constexpr bool ADAPT = (ALG == 4 || ALG == 5);
    constexpr bool NORM = (ALG == 2 || ALG == 4);
    constexpr int S = R + RG;
    static_assert(S <= 64, "VN phase masks are 64-bit");
    // VN terms kk >= vn_k0 through a global stage written by the message pass
    // and summed per bit in one gather pass: the hybrid shape's sparse
    // high-degree terms, and on split frames every term after the first (the
    // totals are global there anyway; the gather reads the stage coalesced).
    static_assert(!VNG || (!SPA_FAM && !SPLIT), "VNG: min-sum family, one workgroup per frame");
    constexpr bool GATHER = (RG > 0 || SPLIT) && !VNG;
    // hybrid bit gather: per-slot padded edge positions in slot_meta2
    constexpr bool VNG_H = VNG && RG > 0;
    constexpr int KT = v2_tail_slots<S>();
    // One-workgroup register frames: the scan takes the row structure from
    // scalar lane masks (a.row_sem) and the row parities from a per-lane
    // decision bit vector (a.row_rmask) instead of per-slot flag bookkeeping;
    // SPA row products are unsigned until their END, where the syndrome sign
    // goes on (sign flips commute with round-to-nearest); min-sum rows get
    // their sign at END and (ANMSA/AOMSA) their mismatch flag after the loop.
    constexpr bool ROWSCAN = V2_ROWSCAN_ON && !SPLIT && RG == 0;

    const int tid = threadIdx.x;
    const int T = a.T, n = a.n, m = a.m, nc = a.nc;
    // threshold_matrix disabled == clipping at +inf (|v| > inf never holds; NaN passes)
    const double thr = a.thr_on ? a.thr : __builtin_inf();
    const double lim = thr < 44.0 ? thr : 44.0;  // SPA: tanh(+-b/2) = +-1 for |b| >= 44, clipped or not
    static_assert(!RGLB || (VNG && RG > 0), "rows in global scratch: hybrid bit gather only");
    static_assert(PL == REG_TSTRIDE || SPLIT, "half-size parts: split frames only");
    const V2Layout L = v2_layout<SPLIT, RL, RGLB, ROWSCAN, R, PL>(a, !SPA_FAM);
    int *s_frame = reinterpret_cast<int *>(smem);
    int *s_flag = reinterpret_cast<int *>(smem) + 1;
    int *s_part = reinterpret_cast<int *>(smem) + 2;  // SPLIT: rank, sync slot
    double *total = reinterpret_cast<double *>(smem + V2_TOTAL_OFF);
    double *const rowA_lds = reinterpret_cast<double *>(smem + L.rows);    // SPA
    double2 *const rowAB_lds = reinterpret_cast<double2 *>(smem + L.rows); // min-sum
    double *rowA = rowA_lds;
    double2 *rowAB = rowAB_lds;
    // RGLB: the leading a.rows_lds layout rows (the rows of waves
    // 0 .. a.rows_lds_waves - 1) stay in LDS, the others live in the
    // workgroup's global scratch.  A wave's scan and message pass touch only
    // its own rows, so there the choice is one scalar branch per access.
    // The global rows are reached by buffer loads / stores only (a pointer
    // select between them and LDS would become flat accesses; a buffer
    // access past the m rows reads 0 and writes nothing).
    const __amdgpu_buffer_rsrc_t rows_rs = __builtin_amdgcn_make_buffer_rsrc(
        RGLB ? (void *)(a.scratch + (size_t)blockIdx.x * a.scratch_wg_doubles + a.rows_wg_offset) : (void *)a.scratch,
        (short)0, RGLB ? a.m * 16 : 0, 0x00020000);
    auto glb_ld = [&](int r) -> double2 { return ld_row16(rows_rs, r); };
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool rows_in_lds = !RGLB || wave < a.rows_lds_waves;
    auto row_ld = [&](int r) -> double2 {
        if constexpr (RGLB) {
            if (rows_in_lds) return rowAB_lds[r];
            return glb_ld(r);
        } else {
            return rowAB[r];
        }
    };
    auto row_st = [&](int r, double2 v) {
        if constexpr (RGLB) {
            if (rows_in_lds) rowAB_lds[r] = v;
            else st_row16(rows_rs, r, v);
        } else {
            rowAB[r] = v;
        }
    };
    double *pal = reinterpret_cast<double *>(smem + V2_PAL_OFF);
    uint8_t *codes = smem + V2_CODES_OFF;
    // total[bit id of metadata word mt] (LDS totals: by col_off8)
    const uint32_t total_lds = (uint32_t)(uintptr_t)(lds_f64 *)(smem + V2_TOTAL_OFF);
    auto tot_at = [&](uint32_t mt) -> auto & {
        if constexpr (!SPLIT) return *col_off8(mt, total_lds);
        else return total[(int)(mt & META_COL_MASK)];
    };

    EdgeMsgsH<R, RG, RL, PL> c2b;
    c2b.bind(a.scratch + (size_t)blockIdx.x * a.scratch_wg_doubles, tid);
    c2b.bind_lds(reinterpret_cast<double *>(smem + L.msl), tid);
    MetaSrcW<S> meta;
    meta.init(a.slot_meta, tid, T);
    // VN phase kk visits only the slots where some lane of this wave holds the
    // kk-th edge of a bit (capi.hip: vn_mask[wave][kk]).
    const uint64_t *vn_mask = a.vn_mask + (size_t)wave * a.dv_max;
    // ... and per slot, the lanes whose edge there is a bit's kk-th: an exec
    // mask loaded by the scalar unit (no per-lane kpos test).
    // (constant address space: read-only for the kernel's lifetime, so the loads are s_load)
    typedef const __attribute__((address_space(4))) uint64_t const_u64;
    const const_u64 *vn_exec = (const const_u64 *)(a.vn_exec + (size_t)wave * a.dv_max * S);
    // SPLIT: this workgroup's XCD (groups never span two L2s)
    uint32_t xcc = 0;
    if constexpr (SPLIT) {
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        xcc &= 15u;
    }
    double *stage = a.scratch + (size_t)blockIdx.x * a.scratch_wg_doubles + a.stage_wg_offset;
    // (only used by the GATHER instantiations; split frames re-point both per frame)
    __amdgpu_buffer_rsrc_t stage_rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)stage, (short)0, GATHER ? 0x7fffffff : 0, 0x00020000);
    __amdgpu_buffer_rsrc_t meta2_rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.slot_meta2, (short)0, (GATHER || VNG) ? S / 4 * REG_TSTRIDE * 16 : 0, 0x00020000);
    const int k0 = GATHER ? a.vn_k0 : (VNG ? 1 : a.dv_max);
    // Per-lane partition constants (capi.hip plan_v2): tail length, first row,
    // rows started here, and the wave's slot count (uniform across the wave).
    const int head_in0 = a.lane_head[tid];
    const int row0_in0 = a.lane_row0[tid];
    const int nst0 = a.lane_nst[tid];
    const int epl0 = __builtin_amdgcn_readfirstlane(a.lane_epl[tid]);
    const int lane = tid & 63;
    const int up = (lane == 0) ? 0 : lane - 1;
    int epoch = 0;
    if (tid == 0) *s_flag = 0;
    // SPA: the expm1 class table of tanh_half_clip_t, once per workgroup (the
    // frame loop's first barrier orders it before any scan)
    // (two arrays of 16-byte entries: A at L.ctab, B right after A)
    // (entries of 32 bytes: A = {X3, X4} then B = {B, C, k << 20}; see exact_math.h)
    ql_exact::Expm1A *const ctab_a = reinterpret_cast<ql_exact::Expm1A *>(smem + L.ctab);
    ql_exact::Expm1B *const ctab_b = reinterpret_cast<ql_exact::Expm1B *>(smem + L.ctab) + 1;
    const ql_exact::Expm1Tab ctab{ctab_a, ctab_b, 2};
    if constexpr (ALG == 0) {
        if (tid < ql_exact::EXPM1_CLASSES)
            ql_exact::expm1_class<SPLIT && QL_SPLIT_TANH_W>(tid + ql_exact::EXPM1_K_MIN, &ctab_a[2 * tid], &ctab_b[2 * tid]);
    }
#ifdef QL_PHASE_STAMPS
    uint64_t st_acc[NUM_STAMPS];
    for (int i = 0; i < NUM_STAMPS; ++i) st_acc[i] = 0;
    uint64_t st_last = __builtin_amdgcn_s_memtime();
#endif

    for (;;) {
        if constexpr (SPLIT) {
            // Claim (slot, rank) on this XCD's counter; rank 0 of a slot draws
            // the frame and publishes it to the slot's other ranks.
            if (tid == 0) {
                const int t = atomicAdd(a.split_claim + xcc, 1);
                const int slot = t / a.split_k, rank = t % a.split_k;
                const int si = (int)xcc * a.split_slots + slot;
                int f = a.batch;
                if (slot < a.split_slots) {
                    int *pub = a.split_pub + si;
                    if (rank == 0) {
                        f = claim_frame(a);
                        __hip_atomic_store(pub, f + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    } else {
                        int v, spins = 0;
                        while ((v = __hip_atomic_load(pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0 &&
                               ++spins < V2_SPLIT_SPIN_LIMIT)
                            __builtin_amdgcn_s_sleep(2);
                        // a group that never forms (cannot happen with >= split_k
                        // workgroups per XCD) is reported, never waited on forever
                        if (v == 0) atomicOr(a.split_err, 1);
                        f = v ? v - 1 : a.batch;
                    }
                }
                *s_frame = f;
                s_part[0] = rank;
                s_part[1] = si;
            }
        } else {
            if (tid == 0) *s_frame = claim_frame(a);
        }
        STAMP(ST_SETUP);
        __syncthreads();
        STAMP(ST_SETUP_WAIT);
        // wave-uniform by construction: readfirstlane lets the compiler keep
        // every per-frame address (llr / stage buffer descriptors) in SGPRs
        // instead of VGPRs with waterfall loops around each access
        const int f = __builtin_amdgcn_readfirstlane(*s_frame);
        if (f >= a.batch) break;
        // SPLIT: this part's lanes, waves, metadata and rows; the group barrier
        const int rank = SPLIT ? __builtin_amdgcn_readfirstlane(s_part[0]) : 0;
        // the trial's own span inside the batch starts at its claim
        // (a.frame_clk; stored now, so no register holds it through the decode)
        if (tid == 0 && rank == 0 && a.frame_clk) a.frame_clk[2 * (size_t)f] = __builtin_amdgcn_s_memrealtime();
        const int tg = SPLIT ? rank * REG_TSTRIDE + tid : tid;
        const int head_in = SPLIT ? a.lane_head[tg] : head_in0;
        const int row0_in = SPLIT ? a.lane_row0[tg] : row0_in0;
        const int nst = SPLIT ? a.lane_nst[tg] : nst0;
        const int epl = SPLIT ? __builtin_amdgcn_readfirstlane(a.lane_epl[tg]) : epl0;
        int gsync_n = 0;
        int *gsync = nullptr, *gmis = nullptr;
        if constexpr (SPLIT) {
            const int si = __builtin_amdgcn_readfirstlane(s_part[1]);
            gsync = a.split_sync + si;
            gmis = a.split_mis + si;
            meta.init(a.slot_meta + (size_t)rank * (S / 4) * REG_TSTRIDE * 4, tid, T);
            const int wg = rank * (REG_TSTRIDE / 64) + wave;
            vn_mask = a.vn_mask + (size_t)wg * a.dv_max;
            vn_exec = (const const_u64 *)(a.vn_exec + (size_t)wg * a.dv_max * S);
            const int rb = a.part_row0[rank];
            rowA = rowA_lds - rb;
            rowAB = rowAB_lds - rb;
            total = a.gtotal + (size_t)f * (n + 1);
            stage = a.gstage + (size_t)f * a.stage_frame_doubles;
            stage_rs = __builtin_amdgcn_make_buffer_rsrc((void *)stage, (short)0, 0x7fffffff, 0x00020000);
            meta2_rs = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(a.slot_meta2 + (size_t)rank * (S / 4) * REG_TSTRIDE * 4), (short)0,
                S / 4 * REG_TSTRIDE * 16, 0x00020000);
        }
        // Phase boundary: the workgroup barrier, or for SPLIT the group's: every
        // wave's global stores reach L2 (the group shares this XCD's L2), one
        // arrival per workgroup, then the frame's totals are re-read past L1.
#define psync()                                                              \
    do {                                                                     \
        if constexpr (SPLIT) {                                               \
            gsync_n += a.split_k;                                            \
            group_sync(gsync, gsync_n, a.split_err);                         \
        } else {                                                             \
            __syncthreads();                                                 \
        }                                                                    \
    } while (0)
        // split frames between a wave's scan and its own message pass
#define split_local_sync()                                                   \
    do {                                                                     \
        if constexpr (SPLIT && QL_SPLIT_DEFER) {                             \
            __syncthreads();                                                 \
        } else {                                                             \
            psync();                                                         \
        }                                                                    \
    } while (0)
        const int bit_lo = SPLIT ? (int)((long long)n * rank / a.split_k) : 0;
        const int bit_hi = SPLIT ? (int)((long long)n * (rank + 1) / a.split_k) : n;
        const uint8_t *sy = a.synd + (size_t)f * m;
        // Target syndrome bits of the rows this lane starts (bit i = i-th START),
        // and of the row it finishes for the lane before (split row).
        // (rows are relabelled by the planner: row_orig maps them back)
        uint32_t smask_f = 0;
        {
            const int rs = row0_in + (head_in > 0 ? 1 : 0);
            for (int i = 0; i < nst; ++i) smask_f |= (uint32_t)(sy[a.row_orig[rs + i]] & 1) << i;
        }
        const int s_row0 = (head_in > 0) ? (sy[a.row_orig[row0_in]] & 1) : 0;
        const bool paletted = a.pal_ok[f] != 0;
        // Non-paletted frames gather llr[] through a buffer resource: a distinct
        // load kind the compiler cannot fuse with the LDS palette read into a
        // flat load.  Relabelled graphs read it by label: such a frame is first
        // copied into label order in this workgroup's scratch (the setup
        // barrier below orders the copy before every read).
        const double *llr_f = a.llr + (size_t)f * n;
        if (!paletted && a.llr_lab_wg_offset >= 0) {
            double *dst = a.scratch + (size_t)blockIdx.x * a.scratch_wg_doubles + a.llr_lab_wg_offset;
            for (int i = tid; i < n; i += T) dst[i] = llr_f[a.col_orig[i]];
            llr_f = dst;
        }
        const __amdgpu_buffer_rsrc_t llr_rs =
            __builtin_amdgcn_make_buffer_rsrc((void *)llr_f, (short)0, paletted ? 0 : n * 8, 0x00020000);
        const uint8_t *gcodes = a.codes + (size_t)f * nc;
        if constexpr (SPLIT) {
            if (tid < 4) pal[tid] = a.palette[(size_t)f * 4 + tid];
        } else if constexpr (VNG) {
            // the per-bit edge-code bytes start cleared (the gather re-clears them)
            uint32_t *codes4 = reinterpret_cast<uint32_t *>(codes);
            for (int i = tid; i < (VNG_H ? V2_CODES_CAP / 4 : nc); i += T) codes4[i] = 0u;
            if (tid < 4) pal[tid] = a.palette[(size_t)f * 4 + tid];
        } else {
            // 2-bit codes -> one byte per bit (the message pass's llr lookup is
            // then a byte read, no shift/mask arithmetic)
            const uint8_t *cs = a.codes + (size_t)f * nc;
            uint32_t *codes4 = reinterpret_cast<uint32_t *>(codes);
            for (int i = tid; i < nc; i += T) {
                const uint32_t b = cs[i];
                codes4[i] = (b & 3u) | (((b >> 2) & 3u) << 8) | (((b >> 4) & 3u) << 16) | ((b >> 6) << 24);
            }
            if (tid < 4) pal[tid] = a.palette[(size_t)f * 4 + tid];
        }
        if constexpr (ROWSCAN) {  // the rows' target syndrome bits as sign words
            uint32_t *syn = reinterpret_cast<uint32_t *>(smem + L.syn);
            for (int r = tid; r < m; r += T) syn[r] = (uint32_t)(sy[a.row_orig[r]] & 1) << 31;
        }
        STAMP(ST_SETUP);
        __syncthreads();
        STAMP(ST_SETUP_WAIT);
        // the frame's 2-bit channel codes by byte buffer loads (32-bit offsets)
        const __amdgpu_buffer_rsrc_t gcodes_rs =
            __builtin_amdgcn_make_buffer_rsrc((void *)gcodes, (short)0, paletted ? nc : 0, 0x00020000);
        auto llr_of = [&](int col) -> double {
            if constexpr (SPLIT || VNG) {
                if (paletted)
                    return pal[((uint32_t)__builtin_amdgcn_raw_buffer_load_b8(gcodes_rs, col >> 2, 0, 0) >> ((col & 3) * 2)) & 3];
            } else {
                if (paletted) return pal[codes[col]];
            }
            // (relabelled graphs: llr_rs holds the frame's label-order copy)
            return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(llr_rs, col * 8, 0, 0));
        };
        // total starts as the channel LLRs: the check-node scan of iteration 0
        // reads the channel decision from it, and bits of degree 0 keep it.
        for (int i = bit_lo + tid; i < bit_hi; i += T) total[i] = llr_of(i);
        if (tid == 0 && rank == 0) total[n] = 1.0;  // dummy column
        // SPA, iteration 0, every channel LLR +-L (the QKD_LDPC frame,
        // src/qkd_ldpc_algorithm.cpp:1043-1052; unused palette entries repeat
        // entry 0): b2c = +-L, so t = +-t0 with t0 = tanh(L / 2.) (tanh is odd
        // in glibc), a row's running product of degree d is +-P_d with P_1 = t0,
        // P_{j+1} = P_j * t0 (the sign of a product never changes its rounding),
        // and every rp / t_k of the row is +-(P_d / t0).  So the iteration's
        // messages are +-A[d], A[d] = clip(2 * atanh(P_d / t0)), computed once
        // per frame by the same functions the general pass calls.
        bool fast0 = false;
        double *const a0tab = reinterpret_cast<double *>(smem + L.a0tab);
        if constexpr (ALG == 0) {
            const double L0 = __builtin_fabs(pal[0]);
            fast0 = paletted && a.max_it > 0 && L0 >= 0x1p-20 && L0 <= 0x1p10 && __builtin_fabs(pal[1]) == L0 &&
                    __builtin_fabs(pal[2]) == L0 && __builtin_fabs(pal[3]) == L0;
            if (fast0 && tid < V2_A0_ENTRIES) {
                int unused = 0;
                const double t0 = ql_exact::tanh_half_clip(L0, 44.0, 1.0, &unused);
                double P = t0;
                for (int j = 1; j < tid; ++j) P = P * t0;
                a0tab[tid] = (tid == 0) ? t0 : ql_exact::atanh2_clip(P / t0, thr, a.spa_ctop);
            }
        }
        STAMP(ST_SETUP);
        psync();
        STAMP(ST_SETUP_WAIT);

        int iters = a.max_it, okv = 0;
        bool had_vn = false;
        // c2b starts at +0: iteration 0's b2c = tv - 0 with the clip at +inf is
        // the channel LLR itself, bitwise (the reference's unclipped
        // initialisation, :21-29), so the scan needs no iteration-0 select
#pragma unroll
        for (int k = 0; k < S; ++k) c2b.set(k, 0.0);
        // Min-sum: after iteration 0 every |b2c| is <= thr, so a message
        // (|c| <= sel when the offset is >= 0 / the factor is <= 1 in
        // magnitude: a.ms_clip_later == 0) needs the clip only when some row
        // kept min2 > thr (rows with < 2 non-NaN b2c): flagged by the scan.
        bool msclip = a.thr_on != 0;
        int *s_big = reinterpret_cast<int *>(smem) + 2;  // (non-split only: s_part's slot)
        // The reference's strict-< two-minimum update (:386-396: ax < m1 ->
        // (ax, m1); else ax < m2 -> (m1, ax)) as min/max: with 0 <= m1 <= m2
        // and ax = |x| >= +0 (no signed zeros), the new m2 is the median
        // max(m1, min(ax, m2)) and the new m1 is min(m1, ax) — ties give
        // equal values, and a NaN ax leaves both unchanged exactly as the
        // reference's false compares do (IEEE minNum / maxNum return the
        // other operand).
        // (v_min/v_max_f64 directly: no input here is a signalling NaN — x
        // comes from arithmetic, m1 / m2 from DBL_MAX and these results — so
        // the compiler's canonicalising copies for fminnum are dropped; |x|
        // is the instructions' abs source modifier, not a separate fabs)
        auto ms_push = [](double &m1, double &m2, double x) {
            double t, u;
            asm("v_min_f64 %0, |%1|, %2" : "=v"(t) : "v"(x), "v"(m2));
            asm("v_max_f64 %0, %1, %2" : "=v"(u) : "v"(m1), "v"(t));
            asm("v_min_f64 %0, %1, |%2|" : "=v"(t) : "v"(m1), "v"(x));
            m2 = u;
            m1 = t;
        };
        auto ms_pack = [](double m1, double m2, int sgn, int mr) -> double2 {
            return make_double2(__builtin_bit_cast(double, __builtin_bit_cast(uint64_t, m1) | ((uint64_t)(sgn & 1) << 63)),
                                __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, m2) | ((uint64_t)(mr & 1) << 63)));
        };
        // Min-sum check-to-bit message of layout row r to an edge whose b2c x
        // has sign bit xneg = (x > 0 ? 0 : 1) and eq1 = (|x| == min1), clipped
        // (:73-74).  Shared by the message pass and the VNG bit gather.
        // Row aggregate {min1, min2} (both >= +0) with the row's sign s xor
        // (parity of negative b2c) in min1's sign bit and its syndrome
        // mismatch (the adaptive factor's selector) in min2's.
        auto ms_message = [&](double2 ab, uint32_t xneg, bool eq1, bool doclip) -> double {
            // sp = (s?-1:1)(-1)^neg (:376,398); prod = sp (x>0?1:-1) (:402): all
            // +-1, and a product by +-1 is a sign flip that commutes with
            // round-to-nearest (signed zeros included), so the reference's
            // fac * prod * sel and prod * max0(d) are computed unsigned and the
            // sign bit goes on by XOR
            const uint32_t sgn = (ql_exact::hi_word(ab.x) ^ (xneg << 31)) & 0x80000000u;
            const double sel = eq1 ? __builtin_fabs(ab.y) : __builtin_fabs(ab.x);  // :406
            double fac = a.primary;
            if (ADAPT && (ql_exact::hi_word(ab.y) >> 31)) fac = a.secondary;  // :749-757
            double c;
            if constexpr (NORM) {
                c = fac * sel;
            } else {
                const double d = sel - fac;
                c = (d < 0.) ? 0. : d;
            }
            c = ql_exact::with_hi_word(c, ql_exact::hi_word(c) ^ sgn);
            if (doclip) {  // (:73-74; a no-op otherwise, see msclip)
                // a real scalar branch on the uniform flag: the empty volatile
                // asm keeps the compiler from turning the clip into selects
                asm volatile("");
                c = clip_msg(c, thr);
            }
            return c;
        };
        // Message emission shared by both message passes: c2b, VN phase 0
        // (total = llr + first message) and the hybrid/split VN stage.
        auto emit = [&](int k, uint32_t mt, uint32_t mt2, double c) {
            c2b.set(k, c);
            const uint32_t kp = (mt >> META_KPOS_SHIFT) & META_KPOS_MASK;
            if constexpr (!SPLIT && !VNG) {
                if (__builtin_amdgcn_inverse_ballot_w64(vn_exec[k])) {  // kpos == 0
                    const int col = (int)(mt & META_COL_MASK);
                    tot_at(mt) = llr_of(col) + c;  // first term of std::accumulate (:78)
                }
            }
            if constexpr (GATHER) {
                if (kp >= (uint32_t)k0 && kp != META_KPOS_MASK) {
                    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, c), stage_rs, (int)(mt2 * 8),
                                                          0, 0);
                }
            }
        };
        // VN phases 1 .. k0-1 and the staged terms (shared by iteration 0's fast path).
        // xchk: split frames' deferred exit test (iteration xchk - 1 ends the
        // decode when no part flagged a mismatch), read past the first
        // barrier; returns true to end it there, before the gather.
        auto vn_phases = [&](int xchk) -> bool {
            STAMP(ST_CN3);
            psync();
            STAMP(ST_VN0_WAIT);
            if constexpr (SPLIT) {
                if (xchk && __hip_atomic_load(gmis, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != xchk) return true;
            }
            // ---- remaining VN phases: the k-th message of every bit, in check order ----
            for (int kk = 1; kk < k0; ++kk) {
                const uint64_t vm = vn_mask[kk];
                const uint32_t mlo = __builtin_amdgcn_readfirstlane((uint32_t)vm);
                const uint32_t mhi = __builtin_amdgcn_readfirstlane((uint32_t)(vm >> 32));
                const const_u64 *ex = vn_exec + (size_t)kk * S;
                // V2_VN_BATCH groups of four slots at a time: their totals are
                // read together by the lanes whose edge there is a kk-th one (a
                // bit's kk-th edge is unique: no two slots of the phase touch
                // one column), then added and written back — one LDS round trip
                // per batch.
                meta.template each_group_batch_masked_pf<V2_VN_BATCH>(mlo, mhi, [&](int g, auto q, int nv) {
                    constexpr int NS = 4 * V2_VN_BATCH;
                    // the lane masks by scalar loads, before any LDS access (a
                    // scalar-load wait also waits for LDS reads)
                    uint64_t em[NS];
#pragma unroll
                    for (int i = 0; i < NS; ++i) em[i] = (i < 4 * nv) ? ex[4 * g + i] : 0ull;
                    double tv[NS];
#pragma unroll
                    for (int i = 0; i < NS; ++i) {
                        // (inactive lanes' tv is never used: the add below runs
                        // under the same mask)
                        asm("" : "=v"(tv[i]));
                        if (i < 4 * nv && __builtin_amdgcn_inverse_ballot_w64(em[i]))
                            tv[i] = tot_at((uint32_t)q[i / 4][i % 4]);
                    }
#pragma unroll
                    for (int i = 0; i < NS; ++i)
                        if (i < 4 * nv && __builtin_amdgcn_inverse_ballot_w64(em[i]))  // kpos == kk
                            tot_at((uint32_t)q[i / 4][i % 4]) =
                                tv[i] + c2b.get((4 * g + i) < S ? 4 * g + i : 0);
                });
                STAMP(ST_VNK);
                psync();
                STAMP(ST_VNK_WAIT);
            }
            if constexpr (VNG_H) {
                // every bit, in degree order (a wave's lanes have similar degree):
                // its messages rebuilt chunk by chunk (four edges: one 8-byte
                // rows load, one code byte) and summed in kpos order onto the
                // channel LLR; a chunk's padding reads row 0 and is not added
                // (two copies of the loop, with and without the clip: the
                // uniform msclip picks one by a scalar branch)
                auto gather_h = [&](auto dct) {
                    constexpr bool DC = decltype(dct)::value;
                    // buffer loads with 32-bit offsets (descriptors in SGPRs)
                    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                    const __amdgpu_buffer_rsrc_t vr_rs =
                        __builtin_amdgcn_make_buffer_rsrc((void *)a.vn_rows, (short)0, 0x7fffffff, 0x00020000);
                    const __amdgpu_buffer_rsrc_t vb_rs =
                        __builtin_amdgcn_make_buffer_rsrc((void *)a.vng_bits, (short)0, n * 8, 0x00020000);
                    auto ld2 = [&](__amdgpu_buffer_rsrc_t rs, uint32_t off) -> uint2 {
                        const u32x2 v = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, (int)off, 0, 0));
                        return make_uint2(v.x, v.y);
                    };
                    // the next bit's entry is requested one bit ahead (its rows
                    // and their aggregates then wait one load each, not two)
                    uint2 e_n = make_uint2(0u, 0u);
                    if (tid < n) e_n = ld2(vb_rs, (uint32_t)tid * 8u);
                    for (int i = tid; i < n; i += T) {
                        const uint2 e = QL_GH_PF ? e_n : ld2(vb_rs, (uint32_t)i * 8u);
                        const int b = (int)e.x;
                        const uint32_t c0 = e.y & 0xFFFFFFu;
                        const int dvb = (int)(e.y >> 24);
                        uint2 rr = ld2(vr_rs, c0 * 8u);
                        if (QL_GH_PF && i + T < n) e_n = ld2(vb_rs, (uint32_t)(i + T) * 8u);
                        double sacc = llr_of(b);
                        for (int kc = 0; kc < dvb; kc += 4) {
                            const uint32_t ch = c0 + (uint32_t)(kc >> 2);
                            const uint2 cur = rr;
                            if (kc + 4 < dvb) rr = ld2(vr_rs, (ch + 1) * 8u);
                            const uint32_t cb = codes[ch];
                            codes[ch] = 0;
                            double2 ab[4];
    #pragma unroll
                            for (int q = 0; q < 4; ++q)
                            {
                                const int rq = (int)(((q < 2 ? cur.x : cur.y) >> (16 * (q & 1))) & 0xFFFFu);
                                if constexpr (RGLB) ab[q] = (rq < a.rows_lds) ? rowAB_lds[rq] : glb_ld(rq);
                                else ab[q] = rowAB[rq];
                            }
    #pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const double c = ms_message(ab[q], (cb >> (2 * q)) & 1u, ((cb >> (2 * q)) & 2u) != 0, DC);
                                sacc = (kc + q < dvb) ? sacc + c : sacc;
                            }
                        }
                        total[b] = sacc;
                    }
                };
                if (msclip) gather_h(std::integral_constant<bool, true>{});
                else gather_h(std::integral_constant<bool, false>{});
                STAMP(ST_VNK);
                psync();
                STAMP(ST_VNK_WAIT);
            } else if constexpr (VNG) {
                // every bit: its dv <= 4 messages rebuilt in kpos order and summed
                // onto the channel LLR.  The next bit's rows and channel code are
                // requested before this bit's work (nothing here waits on them),
                // and a bit's four row aggregates are read together (missing
                // terms read row 0 and are not added).
                auto gather_r = [&](auto dct) {
                    constexpr bool DC = decltype(dct)::value;
                    // buffer loads with 32-bit offsets (descriptors in SGPRs): no
                    // 64-bit address arithmetic per bit
                    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                    const __amdgpu_buffer_rsrc_t vr_rs =
                        __builtin_amdgcn_make_buffer_rsrc((void *)a.vn_rows, (short)0, n * 8, 0x00020000);
                    const __amdgpu_buffer_rsrc_t gc_rs =
                        __builtin_amdgcn_make_buffer_rsrc((void *)gcodes, (short)0, paletted ? nc : 0, 0x00020000);
                    auto ld_rows = [&](int bb) -> uint2 {
                        const u32x2 v = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(vr_rs, bb * 8, 0, 0));
                        return make_uint2(v.x, v.y);
                    };
                    int b = tid;
                    uint2 rr = make_uint2(0u, 0u);
                    uint32_t gcn = 0;
                    double lrn = 0.0;
                    if (b < n) {
                        rr = ld_rows(b);
                        if (paletted) gcn = __builtin_amdgcn_raw_buffer_load_b8(gc_rs, b >> 2, 0, 0);
                        else lrn = llr_of(b);
                    }
                    for (; b < n; b += T) {
                        const uint2 cur = rr;
                        const uint32_t gc = gcn;
                        const double lr = lrn;
                        const int bn = b + T;
                        if (bn < n) {
                            rr = ld_rows(bn);
                            if (paletted) gcn = __builtin_amdgcn_raw_buffer_load_b8(gc_rs, bn >> 2, 0, 0);
                            else lrn = llr_of(bn);
                        }
                        const uint32_t cb = codes[b];
                        codes[b] = 0;
                        uint32_t rk[4];
                        double2 ab[4];
    #pragma unroll
                        for (int kk = 0; kk < 4; ++kk) {
                            rk[kk] = ((kk < 2 ? cur.x : cur.y) >> (16 * (kk & 1))) & 0xFFFFu;
                            ab[kk] = rowAB[rk[kk] != 0xFFFFu ? (int)rk[kk] : 0];
                        }
                        double sacc = paletted ? pal[(gc >> ((b & 3) * 2)) & 3u] : lr;
    #pragma unroll
                        for (int kk = 0; kk < 4; ++kk) {
                            const double c = ms_message(ab[kk], (cb >> (2 * kk)) & 1u, ((cb >> (2 * kk)) & 2u) != 0, DC);
                            sacc = (rk[kk] != 0xFFFFu) ? sacc + c : sacc;
                        }
                        total[b] = sacc;
                    }
                };
                if (msclip) gather_r(std::integral_constant<bool, true>{});
                else gather_r(std::integral_constant<bool, false>{});
                STAMP(ST_VNK);
                psync();
                STAMP(ST_VNK_WAIT);
            }
            if constexpr (SPLIT) {
                if (a.xoff) {
                    // Exchange gather: this part's bits, chunk by chunk, start at
                    // the channel LLR in LDS; then for kpos 0, 1, ... the region
                    // of each kpos is read front to back and every term added at
                    // its bit (one term per bit and kpos: no two lanes of a
                    // phase touch one sum), so each bit's sum runs in kpos order
                    // like std::accumulate (:78); the sums go to the totals.
                    double *const acc = reinterpret_cast<double *>(smem + L.rows);
                    const int D = a.dv_max, NC = a.split_nc, CB = a.split_cb;
                    const __amdgpu_buffer_rsrc_t xb_rs =
                        __builtin_amdgcn_make_buffer_rsrc((void *)a.xbit, (short)0, 0x7fffffff, 0x00020000);
                    constexpr int XU = QL_XG_UNROLL;  // terms per thread per load round
                    for (int c = 0; c < NC; ++c) {
                        const int c0 = bit_lo + c * CB;
                        const int nb = (bit_hi - c0 < CB) ? bit_hi - c0 : CB;
                        for (int i = tid; i < nb; i += T) acc[i] = llr_of(c0 + i);
                        __syncthreads();
                        for (int kk = 0; kk < D; ++kk) {
                            const int rid = (rank * NC + c) * D + kk;
                            const int p0 = __builtin_amdgcn_readfirstlane(a.xoff[rid]);
                            const int p1 = __builtin_amdgcn_readfirstlane(a.xoff[rid + 1]);
                            for (int p = p0 + tid; p < p1; p += XU * T) {
                                uint32_t lb[XU];
                                double v[XU], t[XU];
#pragma unroll
                                for (int j = 0; j < XU; ++j) {
                                    const int q = p + j * T;
                                    lb[j] = 0;
                                    v[j] = 0.0;
                                    if (q < p1) {
                                        lb[j] = __builtin_amdgcn_raw_buffer_load_b16(xb_rs, q * 2, 0, 0);
                                        v[j] = __builtin_bit_cast(
                                            double, __builtin_amdgcn_raw_buffer_load_b64(stage_rs, q * 8, 0, 0));
                                    }
                                }
#pragma unroll
                                for (int j = 0; j < XU; ++j)
                                    if (p + j * T < p1) t[j] = acc[lb[j]];
#pragma unroll
                                for (int j = 0; j < XU; ++j)
                                    if (p + j * T < p1) acc[lb[j]] = t[j] + v[j];
                            }
                            __syncthreads();
                        }
                        // (the next chunk's LLR store hits the same acc[i] from
                        // the same thread: no barrier before it)
                        for (int i = tid; i < nb; i += T) total[c0 + i] = acc[i];
                    }
                    STAMP(ST_VNK);
                    psync();
                    STAMP(ST_VNK_WAIT);
                    return false;
                }
            }
            if constexpr (GATHER) {
                // terms k0 .. dv-1 of each high-degree bit, in order, from the stage
                if (k0 < a.dv_max) {
                    // (split frames: each part sums its share of the bits)
                    const int h0 = SPLIT ? (int)((long long)a.n_hd * rank / a.split_k) : 0;
                    const int h1 = SPLIT ? (int)((long long)a.n_hd * (rank + 1) / a.split_k) : a.n_hd;
                    // four bits per lane at a time: their stage loads overlap
                    for (int i0 = h0 + tid; i0 < h1; i0 += 4 * T) {
                        int b[4], dvb[4];
                        if (a.hd_uniform_dv > 0) {  // regular code, bits in id order: no table loads
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                const int i = i0 + j * T;
                                b[j] = (i < h1) ? i : -1;
                                dvb[j] = (i < h1) ? a.hd_uniform_dv : 0;
                            }
                        } else {
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                const int i = i0 + j * T;
                                b[j] = (i < h1) ? a.hd_bits[i] : -1;
                                dvb[j] = (i < h1) ? a.hd_dv[i] : 0;
                            }
                        }
                        double sacc[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            // split frames stage every term: the sum starts at the channel LLR
                            if constexpr (SPLIT) sacc[j] = (b[j] >= 0) ? llr_of(b[j]) : 0.0;
                            else sacc[j] = (b[j] >= 0) ? total[b[j]] : 0.0;
                        }
                        for (int kk = k0; kk < a.dv_max; ++kk) {
                            const int off = a.stage_off[kk];
                            double v[4];
#pragma unroll
                            for (int j = 0; j < 4; ++j) v[j] = (kk < dvb[j]) ? stage[off + i0 + j * T] : 0.0;
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                if (kk < dvb[j]) sacc[j] = sacc[j] + v[j];
                        }
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (b[j] >= 0) total[b[j]] = sacc[j];
                    }
                    STAMP(ST_VNK);
                    psync();
                    STAMP(ST_VNK_WAIT);
                }
            }
            return false;
        };
        int it0 = 0;
        if (ALG == 0 && fast0) {
            int head = head_in, row0 = row0_in;
            uint32_t sm = smask_f;
            asm volatile("" : "+v"(head), "+v"(row0), "+v"(sm));
            // ---- SPA iteration 0 on a +-L frame (see fast0): t = +-t0, and
            // per row its degree and sign (s xor parity of the negative
            // LLRs = parity of the channel decisions) instead of a product
            int2 *const rowI = reinterpret_cast<int2 *>(rowA);
            const double t0 = a0tab[0];
            int r = row0, par = 0, cnt = 0, cur_s = 0;
            uint32_t zt = 0;
            meta.each_upto(epl, [&](int k, uint32_t mt) {
                const int col = (int)(mt & META_COL_MASK);
                const double tv = total[col];
                const int zb = (tv <= 0.0) ? 1 : 0;
                if (k < KT) zt |= (uint32_t)zb << k;
                const bool start = (mt & META_START) != 0;
                c2b.set(k, __builtin_copysign(t0, tv));
                cur_s = start ? (int)(sm & 1u) : cur_s;
                sm = start ? (sm >> 1) : sm;
                par = (start ? 0 : par) ^ zb;
                cnt = (start ? 0 : cnt) + 1;
                if (k > 0) r += start ? 1 : 0;
                if (mt & META_END) rowI[r] = make_int2(cnt, par ^ cur_s);
            });
            {  // a row split across two lanes of this wave
                const int ppar = __shfl(par, up, 64);
                const int pcnt = __shfl(cnt, up, 64);
                const int hpar = __builtin_popcount(zt & ((1u << head) - 1u)) & 1;
                if (head > 0) rowI[row0] = make_int2(pcnt + head, ppar ^ hpar ^ s_row0);
            }
            STAMP(ST_CN1);
            split_local_sync();  // (no exit test in iteration 0)
            STAMP(ST_CN1_WAIT);
            r = row0;
            auto message0 = [&](int k, uint32_t mt, uint32_t mt2) {
                if (k > 0) r += (mt & META_START) ? 1 : 0;
                const int2 ri = rowI[r];
                const double av = a0tab[ri.x & (V2_A0_ENTRIES - 1)];
                const uint32_t neg = ((uint32_t)ri.y ^ (ql_exact::hi_word(c2b.get(k)) >> 31)) & 1u;
                emit(k, mt, mt2, neg ? -av : av);  // sign of rp / t_k (:66-68)
            };
            if constexpr (GATHER) {
                meta.each_upto2(epl, meta2_rs, message0);
            } else {
                meta.each_upto(epl, [&](int k, uint32_t mt) { message0(k, mt, 0u); });
            }
            vn_phases(0);
            had_vn = true;
            it0 = 1;
        }
        for (int it = it0;; ++it) {
            // SPA: iteration 0's b2c is the unclipped channel LLR (:21-29)
            const double lim_it = had_vn ? lim : 44.0;
            const double tlim_it = had_vn ? a.spa_tlim : 1.0;  // tanh(22) = 1
            const bool check = ADAPT ? (it < a.max_it) : (it > 0);
            const bool compute = it < a.max_it;
            // (iteration 0: b2c unclipped; c2b is +0 there)
            const double thr_it = had_vn ? thr : __builtin_inf();
            ++epoch;
            int head = head_in, row0 = row0_in;
            uint32_t sm = smask_f;
            asm volatile("" : "+v"(head), "+v"(row0), "+v"(sm));

            // ---- check-node scan: b2c, tanh / aggregates, row parity of z ----
            // A START begins a row (bit `sm & 1` of the target syndrome); an END
            // (set only on rows begun in this lane) publishes it.  Slots before
            // the first START are the tail of the previous lane's last row.
            int r = row0;
            int mis = 0, big = 0;
            int div_unsafe = 0;
            if constexpr (ROWSCAN) {
                // Decisions z_k = (total <= 0) are shifted into zA (slots 0..31)
                // and zB (32..), one shift per slot; a row's parity is then the
                // popcount of z under the row's slot mask, after the loop.
                uint32_t zA = 0, zB = 0;
                double acc = 1.0;                      // SPA: running product
                double m1 = DBL_MAX, m2 = DBL_MAX;     // min-sum: aggregate (:381-397)
                int neg = 0;
                const uint32_t *syn = reinterpret_cast<const uint32_t *>(smem + L.syn);
                const cu64_t *sem = (const cu64_t *)(a.row_sem + (size_t)wave * S * 4);
                // slot k's {START, END, PARK} masks are loaded during slot k - 1,
                // after that slot's LDS read is consumed (SMEM and LDS share one
                // wait counter: a scalar load in flight would hold up the LDS wait)
                uint64_t smk = sem[0], emk = sem[1], pmk = sem[2];
                meta.each_upto(epl, [&](int k, uint32_t mt) {
                    const double tv = tot_at(mt);
                    double b;
                    if constexpr (ALG == 0) b = tv - c2b.get(k);  // b2c = total - c2b (:115); +0 in iteration 0
                    else b = clip_msg(tv - c2b.get(k), thr_it);    // (:115, :122-123; :21-29)
                    asm volatile("" ::"v"(b) : "memory");
                    const bool more = k + 1 < S;
                    const uint64_t smk_n = more ? sem[4 * k + 4] : 0, emk_n = more ? sem[4 * k + 5] : 0;
                    const uint64_t pmk_n = (!SPA_FAM && more) ? sem[4 * k + 6] : 0;
                    const bool start = __builtin_amdgcn_inverse_ballot_w64(smk);
                    if (k > 0) r = add_carry(r, 0, smk);  // r += START
                    const uint32_t sv = syn[r];  // sign word of the row this slot belongs to
                    // z = z * 2 + (total <= 0): the compare's lane mask is the carry-in
                    const uint64_t zm = __builtin_amdgcn_ballot_w64(tv <= 0.0);
                    if (k < 32) zA = add_carry(zA, zA, zm);
                    else zB = add_carry(zB, zB, zm);
                    if constexpr (SPA_FAM) {
                        double t = b;
                        if constexpr (ALG == 0) {
                            if (compute) t = ql_exact::tanh_half_clip_t<SPLIT && QL_SPLIT_TANH_W>(b, lim_it, tlim_it, &div_unsafe, ctab);  // (:60)
                        } else {
                            if (compute) t = tanh_lin(b / 2.);
                        }
                        c2b.set(k, t);
                        // running product in CSR order (:57-62), unsigned: the
                        // row's sign (s ? -1 : 1) is applied at its END
                        acc = (start ? 1.0 : acc) * t;
                        if (__builtin_amdgcn_inverse_ballot_w64(emk)) {
                            // two word stores: the low word straight from acc's register
                            uint32_t *ra = reinterpret_cast<uint32_t *>(rowA + r);
                            ra[0] = ql_exact::lo_word(acc);
                            ra[1] = ql_exact::hi_word(acc) ^ sv;
                            if constexpr (ALG == 0) {
                                if (!(__builtin_fabs(acc) >= 0x1p-900)) div_unsafe = 1;
                            }
                        }
                    } else {
                        const double x = b;
                        c2b.set(k, x);
                        // the first START closes the tail segment of a row begun in
                        // the lane before: its aggregate (parity of negatives in
                        // min1's sign bit) is parked in that row's own entry
                        // (the aggregate restarts after a row's END and after the
                        // park — the slot after either is a START — so a START
                        // needs no selects)
                        if (k > 0 && k < KT && __builtin_amdgcn_inverse_ballot_w64(pmk)) {
                            rowAB[row0] = ms_pack(m1, m2, neg, 0);
                            m1 = DBL_MAX;
                            m2 = DBL_MAX;
                            neg = 0;
                        }
                        // agg_push (:381-397), branch-free; the count of negatives
                        // by v_addc (only its parity bit is ever read)
                        neg = add_carry(neg, 0, __builtin_amdgcn_ballot_w64(x < 0));
                        ms_push(m1, m2, x);
                        if (__builtin_amdgcn_inverse_ballot_w64(emk)) {
                            // s xor parity(negatives) in min1's sign; the mismatch
                            // flag (ANMSA/AOMSA) is set after the loop
                            rowAB[r] = ms_pack(m1, m2, neg ^ (int)(sv >> 31), 0);
                            big |= (m2 > thr) ? 1 : 0;
                            m1 = DBL_MAX;
                            m2 = DBL_MAX;
                            neg = 0;
                        }
                    }
                    smk = smk_n;
                    emk = emk_n;
                    pmk = pmk_n;
                });
                // bit k of (zlo, zhi) = decision of slot k
                const int na = epl < 32 ? epl : 32;
                const uint32_t zlo = __builtin_bitreverse32(zA) >> (32 - na);
                const uint32_t zhi = (epl > 32) ? (__builtin_bitreverse32(zB) >> (64 - epl)) : 0u;
                // rows started in this lane: parity of the decisions under the
                // row's slots vs its target syndrome bit (sm: bit j = j-th START)
                int popen = 0;
                const int rs0 = row0 + (head > 0 ? 1 : 0);
                for (int j = 0; j < a.nst_max; ++j) {
                    if (j < nst) {
                        const uint64_t mk = a.row_rmask[(size_t)j * T + tid];
                        const int p = (__builtin_popcount(zlo & (uint32_t)mk) +
                                       __builtin_popcount(zhi & (uint32_t)(mk >> 32) & 0x7fffffffu)) & 1;
                        if (mk >> 63) {
                            popen = p;  // continues in the next lane
                        } else {
                            const int mr = p ^ (int)((sm >> j) & 1u);
                            mis |= mr;
                            if constexpr (ADAPT) {  // factor selector in min2's sign bit (:749-757)
                                if (mr) reinterpret_cast<uint32_t *>(rowAB + rs0 + j)[3] |= 0x80000000u;
                            }
                        }
                    }
                }
                // a row split across two lanes of this wave: finished here
                const int ppar = __shfl(popen, up, 64);
                const int hpar = __builtin_popcount(zlo & ((1u << head) - 1u)) & 1;
                if constexpr (SPA_FAM) {
                    const double pacc = __shfl(acc, up, 64);
                    if (head > 0) {
                        double p = pacc;  // continue the row's product in CSR order
#pragma unroll
                        for (int k = 0; k < KT; ++k)
                            if (k < head) p = p * c2b.get(k);
                        rowA[row0] = ql_exact::with_hi_word(p, ql_exact::hi_word(p) ^ syn[row0]);
                        if constexpr (ALG == 0) div_unsafe |= (__builtin_fabs(p) >= 0x1p-900) ? 0 : 1;
                        mis |= ppar ^ hpar ^ s_row0;
                    }
                } else {
                    MinAgg t;
                    t.m1 = __shfl(m1, up, 64);
                    t.m2 = __shfl(m2, up, 64);
                    t.neg = __shfl(neg, up, 64);
                    if (head > 0) {
                        const double2 ta = rowAB[row0];
                        MinAgg h;
                        h.m1 = __builtin_fabs(ta.x);
                        h.m2 = ta.y;
                        h.neg = (int)(ql_exact::hi_word(ta.x) >> 31);
                        agg_merge(t, h);
                        const int mr = ppar ^ hpar ^ s_row0;
                        rowAB[row0] = ms_pack(t.m1, t.m2, s_row0 ^ t.neg, mr);
                        big |= (t.m2 > thr) ? 1 : 0;
                        mis |= mr;
                    }
                }
            } else {
            int par = 0, cur_s = 0, neg = 0;
            uint32_t zt = 0;  // decisions of the first KT slots (tail parity)
            double acc = 1.0, m1 = DBL_MAX, m2 = DBL_MAX;
            auto scan_slot = [&](int k, uint32_t mt, double tv) {
                const int zb = (tv <= 0.0) ? 1 : 0;
                if (k < KT) zt |= (uint32_t)zb << k;
                const bool start = (mt & META_START) != 0;
                const int s = (int)(sm & 1u);
                if constexpr (ALG == 0) {
                    // b2c = total - c2b (:115); c2b is +0 in iteration 0, so b = the
                    // channel LLR exactly there, and the clip (:122-123) is folded
                    // into tanh_half_clip with the iteration's (lim, thr).
                    const double b = tv - c2b.get_seq(k);
                    double t = b;
                    if (compute) t = ql_exact::tanh_half_clip_t<SPLIT && QL_SPLIT_TANH_W>(b, lim_it, tlim_it, &div_unsafe, ctab);  // tanh(b2c / 2.) (:60)
                    c2b.set(k, t);
                    const double st = (s ? -1. : 1.) * t;  // (:57-62)
                    acc = start ? st : acc * t;
                } else if constexpr (SPA_FAM) {
                    const double x = clip_msg(tv - c2b.get_seq(k), thr_it);  // (:115, :122-123; :21-29)
                    double t = x;
                    if (compute) t = tanh_lin(x / 2.);
                    c2b.set(k, t);
                    const double st = (s ? -1. : 1.) * t;  // (:57-62)
                    acc = start ? st : acc * t;
                } else {
                    const double x = clip_msg(tv - c2b.get_seq(k), thr_it);  // (:115, :122-123; :21-29)
                    c2b.set(k, x);
                    if (k < KT && k > 0) {
                        // the first START closes the tail segment: park its aggregate
                        // (parity of negatives in min1's sign bit) in the split row's
                        // own entry, which nothing else touches until the merge below
                        if (k == head) row_st(row0, ms_pack(m1, m2, neg, 0));
                    }
                    m1 = start ? DBL_MAX : m1;
                    m2 = start ? DBL_MAX : m2;
                    neg = start ? 0 : neg;
                    // agg_push (:381-397), branch-free
                    neg ^= (x < 0) ? 1 : 0;
                    ms_push(m1, m2, x);
                }
                cur_s = start ? s : cur_s;
                sm = start ? (sm >> 1) : sm;
                par = (start ? 0 : par) ^ zb;
                if (k > 0) r += start ? 1 : 0;
                if (mt & META_END) {
                    const int mr = par ^ cur_s;
                    mis |= mr;
                    if constexpr (SPA_FAM) {
                        rowA[r] = acc;
                        if constexpr (ALG == 0) div_unsafe |= (__builtin_fabs(acc) >= 0x1p-900) ? 0 : 1;
                    } else {
                        row_st(r, ms_pack(m1, m2, cur_s ^ neg, mr));
                        big |= (m2 > thr) ? 1 : 0;
                    }
                }
            };
            if constexpr (SPLIT) {  // totals in global memory: a group's four loads issued together
#ifdef QL_DIAG_SCAN_HOT  // (diagnostic A/B only: every total read from 256 L1-hot entries — wrong decodes)
                meta.each_upto_tv(epl, [&](uint32_t mt) { return total[(int)(mt & 255)]; }, scan_slot);
#else
                meta.each_upto_tv(epl, [&](uint32_t mt) { return total[(int)(mt & META_COL_MASK)]; }, scan_slot);
#endif
            } else {
                meta.each_upto(epl, [&](int k, uint32_t mt) { scan_slot(k, mt, tot_at(mt)); });
            }
            // ---- rows split across two lanes of this wave: one shuffle ----
            {
                const int ppar = __shfl(par, up, 64);
                const int hpar = __builtin_popcount(zt & ((1u << head) - 1u)) & 1;
                if constexpr (SPA_FAM) {
                    const double pacc = __shfl(acc, up, 64);
                    if (head > 0) {
                        double p = pacc;  // continue the row's product in CSR order
#pragma unroll
                        for (int k = 0; k < KT; ++k)
                            if (k < head) p = p * c2b.get(k);
                        rowA[row0] = p;
                        if constexpr (ALG == 0) div_unsafe |= (__builtin_fabs(p) >= 0x1p-900) ? 0 : 1;
                        mis |= ppar ^ hpar ^ s_row0;
                    }
                } else {
                    MinAgg t;
                    t.m1 = __shfl(m1, up, 64);
                    t.m2 = __shfl(m2, up, 64);
                    t.neg = __shfl(neg, up, 64);
                    if (head > 0) {
                        const double2 ta = row_ld(row0);
                        MinAgg h;
                        h.m1 = __builtin_fabs(ta.x);
                        h.m2 = ta.y;
                        h.neg = (int)(ql_exact::hi_word(ta.x) >> 31);
                        agg_merge(t, h);
                        const int mr = ppar ^ hpar ^ s_row0;
                        row_st(row0, ms_pack(t.m1, t.m2, s_row0 ^ t.neg, mr));
                        big |= (t.m2 > thr) ? 1 : 0;
                        mis |= mr;
                    }
                }
            }
            }  // !ROWSCAN
            if constexpr (SPLIT) {
                if (mis) __hip_atomic_store(gmis, it + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                if (mis) *s_flag = epoch;
                if constexpr (!SPA_FAM) {
                    if (big) *s_big = epoch;
                }
            }
            STAMP(ST_CN1);
            // Split frames defer the exit test past the message pass (it writes
            // only the stage: the totals the outputs read are untouched), to
            // the barrier before the gather: one group barrier per iteration
            // fewer, one wasted message pass on the last.  The message pass
            // reads only rows its own wave scanned.
            const bool defer = SPLIT && QL_SPLIT_DEFER && compute;
            if (defer) split_local_sync();
            else psync();
            STAMP(ST_CN1_WAIT);
            const bool anymis =
                defer || (SPLIT ? (__hip_atomic_load(gmis, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == it + 1)
                                : (*s_flag == epoch));
            if constexpr (!SPA_FAM)
                msclip = a.thr_on && (SPLIT || !had_vn || a.ms_clip_later || *s_big == epoch);
            // SPA: rp / t by div_rn_safe when every t of this wave came out of
            // tanh's common path (|t| in [2^-55, 1]) and every row product of the
            // wave is at least 2^-900 in magnitude: the operand range where the
            // shortened Newton sequence is the IEEE quotient (exact_math.h).
            const bool div_fast = (ALG == 0) && !__builtin_amdgcn_ballot_w64(div_unsafe != 0);
            if (check && !anymis) {
                iters = ADAPT ? it + 1 : it;
                okv = 1;
                break;
            }
            if (!compute) break;

            // ---- check-to-bit messages + VN phase 0 (total = llr + first message) ----
            // RGLB: a wave whose rows live in global scratch copies them (just
            // written by its own scan) into the totals region, which nothing
            // reads until the bit gather rewrites it: its messages then read
            // LDS.  A wave's message pass touches only its own rows, so no
            // barrier; the gather still reads these rows from global.
            // (row r >= rows_lds at rowcopy[r - rows_lds]: indices, never a
            // pointer below the LDS block)
            double2 *const rowcopy = reinterpret_cast<double2 *>(smem + V2_TOTAL_OFF);
            if constexpr (RGLB) {
                if (!rows_in_lds && a.rows_copy) {
                    const int r0 = __builtin_amdgcn_readfirstlane(a.wave_rows[wave]);
                    const int r1 = __builtin_amdgcn_readfirstlane(a.wave_rows[wave + 1]);
                    for (int rr = r0 + lane; rr < r1; rr += 64) rowcopy[rr - a.rows_lds] = glb_ld(rr);
                }
            }
            // (wave-uniform: the message pass's rows, one LDS pointer or L2)
            const bool msg_glb = RGLB && !rows_in_lds && !a.rows_copy;
            double2 *const rows_msg = (RGLB && !rows_in_lds) ? rowcopy : rowAB_lds;
            const int msg_off = (RGLB && !rows_in_lds) ? a.rows_lds : 0;
            r = row0;
            // SPA on ROWSCAN shapes: the row counter by the scalar START mask
            // (v_addc; the min-sum message pass is too short to hide the load)
            const cu64_t *sem_m = ROWSCAN ? (const cu64_t *)(a.row_sem + (size_t)wave * S * 4) : nullptr;
            auto message = [&](int k, uint32_t mt, uint32_t mt2) {
                if constexpr (ROWSCAN && SPA_FAM) {
                    if (k > 0) r = add_carry(r, 0, sem_m[4 * k]);
                } else {
                    if (k > 0) r += (mt & META_START) ? 1 : 0;
                }
                double c;
                // SPA on one-workgroup register shapes: a kpos-0 edge's channel
                // LLR (two dependent LDS reads) is requested before the message
                // math, so its latency hides behind it (VN phase 0 below)
                constexpr bool HOIST = QL_HOIST_LLR && ALG == 0 && !SPLIT && !VNG && !GATHER;
                bool kpos0 = false;
                double lv0 = 0.0;
                if constexpr (HOIST) {
                    kpos0 = __builtin_amdgcn_inverse_ballot_w64(vn_exec[k]);
                    if (kpos0) lv0 = llr_of((int)(mt & META_COL_MASK));
                }
                if constexpr (ALG == 0) {
                    // 2. * atanh(rp / t) (:66-68) and the clip (:73-74) in one
                    const double ra = rowA[r], tk = c2b.get_seq(k);
                    double prod;  // :66
                    if (div_fast) prod = ql_exact::div_rn_safe(ra, tk);
                    else prod = ra / tk;
                    c = ql_exact::atanh2_clip(prod, thr, a.spa_ctop);
                } else if constexpr (SPA_FAM) {
                    const double prod = rowA[r] / c2b.get_seq(k);  // :66
                    c = 2. * atanh_lin(prod);
                } else {
                    const double x = c2b.get_seq(k);
                    const uint32_t xneg = (x > 0) ? 0u : 1u;
                    // the two recorded bits: xneg | eq1 << 1, as one v_addc with
                    // the xneg lane mask as carry-in (no select + or)
                    auto rec2 = [&](bool eq1) -> uint32_t {
                        return add_carry(eq1 ? 2u : 0u, 0u, __builtin_amdgcn_ballot_w64(!(x > 0)));
                    };
                    double2 ab;
                    // (lanes without edges may hold any row: the index is clamped)
                    if constexpr (RGLB) ab = msg_glb ? glb_ld(r) : rows_msg[max(r - msg_off, 0)];
                    else ab = row_ld(r);
                    const bool eq1 = __builtin_fabs(x) == __builtin_fabs(ab.x);
                    c = ms_message(ab, xneg, eq1, msclip);
                    if constexpr (VNG_H) {
                        // the two bits at the edge's padded position (dummy slots:
                        // a scratch byte past the last chunk)
                        __hip_atomic_fetch_or(reinterpret_cast<uint32_t *>(codes) + (mt2 >> 4),
                                              rec2(eq1) << ((mt2 & 15u) * 2),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else if constexpr (VNG) {
                        // record the two bits the bit gather rebuilds this message
                        // from, at the word and shift the host precomputed (mt2;
                        // dummy slots: the spare word past the codes, never read)
                        __hip_atomic_fetch_or(reinterpret_cast<uint32_t *>(codes + (mt2 & 0xFFFFu)),
                                              rec2(eq1) << (mt2 >> 16),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                if constexpr (SPA_FAM && ALG != 0) c = clip_msg(c, thr);  // (:73-74)
                if constexpr (HOIST) {
                    c2b.set(k, c);
                    if (kpos0) tot_at(mt) = lv0 + c;  // first term of std::accumulate (:78)
                } else {
                    emit(k, mt, mt2, c);
                }
            };
            if constexpr (GATHER && QL_MSG_PF) {  // (global stage stores per slot)
                meta.each_upto2_pf(epl, meta2_rs, message);
            } else if constexpr (GATHER || VNG) {
                meta.each_upto2(epl, meta2_rs, message);
            } else {
                meta.each_upto(epl, [&](int k, uint32_t mt) { message(k, mt, 0u); });
            }
            if (vn_phases(defer && check ? it + 1 : 0)) {
                iters = ADAPT ? it + 1 : it;
                okv = 1;
                break;
            }
            had_vn = true;
        }

        // ---- outputs ----
        // ANMSA/AOMSA's total_bit_llr starts zeroed (:738): posterior 0 when the
        // channel decision already satisfied the syndrome.
        const bool zero_post = ADAPT && !had_vn;
        uint8_t *bits = a.bits + (size_t)f * n;
        double *post = a.post ? a.post + (size_t)f * n : nullptr;
        // (relabelled graphs: bit i's total sits at its label)
        const int32_t *const clab = a.col_lab;
        for (int i = bit_lo + tid; i < bit_hi; i += T) {
            const double z = total[clab ? clab[i] : i];
            bits[i] = (z <= 0.0) ? 1 : 0;
            if (post) post[i] = zero_post ? 0.0 : z;
        }
        if (tid == 0 && rank == 0) {
            a.iters[f] = (uint32_t)iters;
            a.ok[f] = (uint8_t)okv;
            if (a.frame_clk) a.frame_clk[2 * (size_t)f + 1] = __builtin_amdgcn_s_memrealtime();
        }
        STAMP(ST_OUT);
        __syncthreads();
        STAMP(ST_OUT_WAIT);
    }
#ifdef QL_PHASE_STAMPS
    if ((tid & 63) == 0 && a.stamps) {
        uint64_t *dst = a.stamps + ((size_t)blockIdx.x * (a.T / 64) + (tid >> 6)) * NUM_STAMPS;
        for (int i = 0; i < NUM_STAMPS; ++i) dst[i] = st_acc[i];
    }
#endif
}
#undef psync
#undef split_local_sync

// Palette + 2-bit codes of each frame's LLRs (one workgroup per frame).  Wave 0
// collects up to 4 distinct values (bitwise) in first-occurrence order; a frame
// with more gets pal_ok = 0 and the decoder gathers its llr[] instead.  Unused
// entries repeat entry 0 (the SPA iteration-0 test reads all four).
__global__ void __launch_bounds__(256) palettize_kernel(int n, int nc, const double *llr, uint8_t *codes,
                                                        double *palette, uint8_t *pal_ok, const int32_t *col_orig) {
    __shared__ unsigned long long pv[4];
    __shared__ int pcount, over;
    const size_t f = blockIdx.x;
    const unsigned long long *v = reinterpret_cast<const unsigned long long *>(llr + f * (size_t)n);
    if (threadIdx.x < 64) {
        int cnt = 0;
        unsigned long long p[4] = {0, 0, 0, 0};
        bool overflow = false;
        for (int base = 0; base < n && !overflow; base += 64) {
            const int i = base + threadIdx.x;
            const unsigned long long x = (i < n) ? v[i] : p[0];
            bool known = (i >= n);
            for (int q = 0; q < 4; ++q) known |= (q < cnt) && (x == p[q]);
            unsigned long long pending = __ballot(!known);
            while (pending) {
                if (cnt == 4) { overflow = true; break; }
                const int src = __builtin_ctzll(pending);
                const unsigned long long nv = __shfl(x, src, 64);
                p[cnt++] = nv;
                known |= (x == nv);
                pending = __ballot(!known);
            }
        }
        if (threadIdx.x == 0) {
            for (int q = 0; q < 4; ++q) pv[q] = (q < cnt) ? p[q] : p[0];  // unused entries repeat entry 0
            pcount = cnt;
            over = overflow ? 1 : 0;
        }
    }
    __syncthreads();
    const int cnt = pcount;
    if (threadIdx.x < 4) palette[f * 4 + threadIdx.x] = __builtin_bit_cast(double, pv[threadIdx.x]);
    if (threadIdx.x == 0) pal_ok[f] = over ? 0 : 1;
    uint8_t *cs = codes + f * (size_t)nc;
    for (int j = threadIdx.x; j < nc; j += blockDim.x) {
        int byte = 0;
        for (int s = 0; s < 4; ++s) {
            const int i = 4 * j + s;  // a label (col_orig: the codes are in label order)
            int code = 0;
            if (i < n) {
                const unsigned long long x = v[col_orig ? col_orig[i] : i];
                for (int q = 1; q < 4; ++q)
                    if (q < cnt && x == pv[q]) code = q;
            }
            byte |= code << (2 * s);
        }
        cs[j] = (uint8_t)byte;
    }
}

using KernelFn = void (*)(DecodeArgs);

template <int R, int RG, bool SPLIT = false, int PL = REG_TSTRIDE>
KernelFn pick_v2(int alg) {
    switch (alg) {
    case 0: return decode_v2_kernel<0, R, RG, SPLIT, 0, false, false, PL>;
    case 1: return decode_v2_kernel<1, R, RG, SPLIT, 0, false, false, PL>;
    case 2: return decode_v2_kernel<2, R, RG, SPLIT, 0, false, false, PL>;
    case 3: return decode_v2_kernel<3, R, RG, SPLIT, 0, false, false, PL>;
    case 4: return decode_v2_kernel<4, R, RG, SPLIT, 0, false, false, PL>;
    default: return decode_v2_kernel<5, R, RG, SPLIT, 0, false, false, PL>;
    }
}

KernelFn kernel_v2_vng(int alg, int RG, bool rglb) {
    if (RG > 0 && rglb) {
        switch (alg) {
        case 2: return decode_v2_kernel<2, V2_R_SMALL, V2_RG_HYBRID, false, 0, true, true>;
        case 3: return decode_v2_kernel<3, V2_R_SMALL, V2_RG_HYBRID, false, 0, true, true>;
        case 4: return decode_v2_kernel<4, V2_R_SMALL, V2_RG_HYBRID, false, 0, true, true>;
        default: return decode_v2_kernel<5, V2_R_SMALL, V2_RG_HYBRID, false, 0, true, true>;
        }
    }
    if (RG > 0) {
        switch (alg) {
        case 2: return decode_v2_kernel<2, V2_R_SMALL, V2_RG_HYBRID, false, 0, true>;
        case 3: return decode_v2_kernel<3, V2_R_SMALL, V2_RG_HYBRID, false, 0, true>;
        case 4: return decode_v2_kernel<4, V2_R_SMALL, V2_RG_HYBRID, false, 0, true>;
        default: return decode_v2_kernel<5, V2_R_SMALL, V2_RG_HYBRID, false, 0, true>;
        }
    }
    switch (alg) {
    case 2: return decode_v2_kernel<2, V2_R_TIGHT, 0, false, 0, true>;
    case 3: return decode_v2_kernel<3, V2_R_TIGHT, 0, false, 0, true>;
    case 4: return decode_v2_kernel<4, V2_R_TIGHT, 0, false, 0, true>;
    default: return decode_v2_kernel<5, V2_R_TIGHT, 0, false, 0, true>;
    }
}

// Split frames: parts of 16 or 8 waves (PL lanes), SG scratch slots (0 or V2_RG_SPLIT).
template <int SG, int PL>
KernelFn kernel_split(int alg, bool rl) {
    constexpr int RL = v2_rl_split(PL);
    if (rl) return alg == 0 ? decode_v2_kernel<0, V2_R_SPLIT, SG, true, RL, false, false, PL>
                            : decode_v2_kernel<1, V2_R_SPLIT, SG, true, RL, false, false, PL>;
    return pick_v2<V2_R_SPLIT, SG, true, PL>(alg);
}

KernelFn kernel_v2(int R, int RG, int split_k, int alg, bool rl, int pl = REG_TSTRIDE) {
    if (split_k > 1) {
        if (RG != 0 && RG != V2_RG_SPLIT) return nullptr;  // (no such instantiation)
        if (pl == REG_TSTRIDE / 2)
            return RG ? kernel_split<V2_RG_SPLIT, REG_TSTRIDE / 2>(alg, rl) : kernel_split<0, REG_TSTRIDE / 2>(alg, rl);
        return RG ? kernel_split<V2_RG_SPLIT, REG_TSTRIDE>(alg, rl) : kernel_split<0, REG_TSTRIDE>(alg, rl);
    }
    if (rl) return alg == 0 ? decode_v2_kernel<0, V2_R_TIGHT, 0, false, V2_RL> : decode_v2_kernel<1, V2_R_TIGHT, 0, false, V2_RL>;
    if (RG > 0) return pick_v2<V2_R_SMALL, V2_RG_HYBRID>(alg);
    if (R == V2_R_TIGHT) return pick_v2<V2_R_TIGHT, 0>(alg);
    if (R == V2_R_SMALL) return pick_v2<V2_R_SMALL, 0>(alg);
    return pick_v2<V2_R_MID, 0>(alg);
}

}  // namespace

size_t lds_bytes_v2(int alg, int n, int m, int T, bool split, int R, int RG, int rows_lds, int gcb) {
    if (split)  // (T: the part's lanes)
        return V2Layout(n, m, (n + 3) / 4, T, alg >= 2, true, v2_use_rl_split(alg, n, m, gcb, T) ? v2_rl_split(T) : 0,
                        false, gcb, T)
            .bytes;
    const bool rl = v2_use_rl(alg, R, RG, split, n, m, T);
    return V2Layout(n, rows_lds >= 0 ? rows_lds : m, (n + 3) / 4, T, alg >= 2, split, rl ? V2_RL : 0,
                    V2_ROWSCAN_ON && !split && RG == 0).bytes;
}

bool v2_split_rl_fits(int n, int mrows, int gcb, int pl) { return v2_use_rl_split(0, n, mrows, gcb, pl); }

bool v2_vng_ok(int alg, int R, int RG, int split_k, int dv_max, int m) {
    if (alg < 2 || split_k > 1 || m >= 0xFFFF) return false;
    if (RG == 0) return R == V2_R_TIGHT && dv_max <= 4;
    return R == V2_R_SMALL && RG == V2_RG_HYBRID;  // + the host's LDS fit test
}

// Every one-workgroup register shape gets row_sem from the planner only when
// its slot count fits the 63 slot bits of a row mask (capi.hip build_meta):
// a larger shape would plan and then fail every launch below.
static_assert(V2_R_TIGHT <= 63 && V2_R_SMALL <= 63 && V2_R_MID <= 63,
              "register shapes without RG slots must have <= 63 slots (row_sem / row_rmask)");

hipError_t launch_decode_v2(const DecodeArgs &a, int workgroups, size_t lds_bytes, hipStream_t stream) {
    // the scan of one-workgroup register frames reads the row structure masks
    // (plan_v2 only builds register shapes of <= 63 slots, which always get row_sem)
    if (a.split_k <= 1 && a.v2RG == 0 && !a.row_sem) return hipErrorInvalidValue;
    if (a.split_k <= 1 && a.n >= 0xFFFF) return hipErrorInvalidValue;  // col_off8: LDS totals, bit ids < 2^16
    if (a.vn_rows && !v2_vng_ok(a.alg, a.v2R, a.v2RG, a.split_k, a.dv_max, a.m)) return hipErrorInvalidValue;
    if (a.rows_wg_offset >= 0 && !(a.vn_rows && a.v2RG > 0)) return hipErrorInvalidValue;
    KernelFn k = a.vn_rows ? kernel_v2_vng(a.alg, a.v2RG, a.rows_wg_offset >= 0)
                           : kernel_v2(a.v2R, a.v2RG, a.split_k, a.alg,
                                       a.split_k > 1 ? v2_use_rl_split(a.alg, a.n, a.split_mrows, a.split_cb, a.T)
                                                     : v2_use_rl(a.alg, a.v2R, a.v2RG, false, a.n, a.m, a.T),
                                       a.split_k > 1 ? a.T : REG_TSTRIDE);
    if (!k) return hipErrorInvalidValue;
    if (a.split_k > 1 && a.T != REG_TSTRIDE && a.T != REG_TSTRIDE / 2) return hipErrorInvalidValue;
    hipError_t e = allow_dynamic_lds(reinterpret_cast<const void *>(k), lds_bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(workgroups), dim3(a.T), lds_bytes, stream, a);
    return hipGetLastError();
}

hipError_t occupancy_v2(int R, int RG, int split_k, int alg, int T, size_t lds_bytes, int *blocks_per_cu) {
    KernelFn k = kernel_v2(R, RG, split_k, alg, false, split_k > 1 ? T : REG_TSTRIDE);
    if (!k) return hipErrorInvalidValue;
    hipError_t e = allow_dynamic_lds(reinterpret_cast<const void *>(k), lds_bytes);
    if (e != hipSuccess) return e;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k, T, lds_bytes);
}

hipError_t launch_palettize(int n, int nc, int batch, const double *llr, uint8_t *codes, double *palette,
                            uint8_t *pal_ok, const int32_t *col_orig, hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    hipLaunchKernelGGL(palettize_kernel, dim3(batch), dim3(256), 0, stream, n, nc, llr, codes, palette, pal_ok,
                       col_orig);
    return hipGetLastError();
}

}  // namespace qldpc
