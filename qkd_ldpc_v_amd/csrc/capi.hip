// capi.hip — the C ABI of libqkdldpc_hip.so (include/qkd_ldpc_hip.h).
//
// Graph planning: the Tanner graph of H (the reference's H_matrix,
// src/array_and_matrix_operations.hpp:60-77) is turned once into the decoder's
// lane partition — E edges in CSR order dealt EPL-per-lane to T lanes — plus a
// row-ELL copy for syndrome checks, and replicated on each device of the
// graph.  Decoding is the persistent kernel of decoder.hip; the host-buffer
// entry shards frames over devices (one host thread per device, contiguous
// slices, no collectives) — the multi-GPU analogue of the reference's
// BS::thread_pool over trials (src/simulation.cpp:721,740-746).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <random>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/qkd_ldpc_hip.h"
#include "decoder.hpp"
#include "loaders.hpp"
#include "relabel.hpp"

using namespace qldpc;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}
int hip_fail(hipError_t e, const char *what) {
    return fail(QLDPC_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr)                                         \
    do {                                                      \
        hipError_t _e = (expr);                               \
        if (_e != hipSuccess) return hip_fail(_e, #expr);     \
    } while (0)

constexpr size_t LDS_LIMIT = 160 * 1024;

struct Workspace {  // per (device, stream): frame counter + decoder scratch
    int *counter = nullptr;
    double *scratch = nullptr;
    size_t scratch_doubles = 0;
    // V2 frame format (palette + 2-bit codes), capacity in frames
    uint8_t *codes = nullptr, *pal_ok = nullptr;
    double *palette = nullptr;
    size_t code_frames = 0;
    // V2 split frames: group claim / publish / barrier / mismatch slots and the
    // frames' totals, capacity in frames
    int *split_ctl = nullptr;
    double *gtotal = nullptr, *gstage = nullptr;
    size_t split_frames = 0;
    // frame claim order (order.hip): per-frame weights and the sorted order
    int32_t *fweight = nullptr, *forder = nullptr;
    size_t order_frames = 0;
    int order_count = 0;  // frames of the last decode claimed through forder (0: index order)
    // the fused entries' frame LLRs when the caller passes no workspace and the
    // graph's decoder reads llr[] (not V2), capacity in frames
    double *llr_ws = nullptr;
    size_t llr_ws_frames = 0;
    // kernel timing (qldpc_set_kernel_timing): events around the last decode launch
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool ev_recorded = false;
};

struct HostIO {  // device staging buffers of the host-buffer entry
    double *llr = nullptr, *post = nullptr;
    uint8_t *synd = nullptr, *bits = nullptr, *ok = nullptr;
    uint32_t *iters = nullptr;
    size_t cap_frames = 0;
    hipStream_t stream = nullptr;
};

// qldpc_run_trials: one pipeline slot of a device's trial batches — the
// chunk's seeds, keys and results on device, its results in pinned host memory
// (two slots per device: chunk c + 1's trials are generated while chunk c
// decodes on the other stream).
struct TrialSlot {
    hipStream_t stream = nullptr;
    // the chunk's window: from ev0 (after its trials are generated) or the end
    // of the other slot's chunk before it (prev_end), whichever is later, to
    // ev1 (after the key compare).  ev1 alternates over ev_end, so the other
    // slot's next chunk never re-records the end a window is measured from.
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_end[2] = {nullptr, nullptr}, prev_end = nullptr;
    int ev_i = 0;
    uint64_t *seeds = nullptr, *clk = nullptr;
    uint8_t *alice = nullptr, *bob = nullptr, *palice = nullptr, *pbob = nullptr, *alice_ext = nullptr;
    uint8_t *synd = nullptr, *bits = nullptr, *ok = nullptr, *km = nullptr;
    uint32_t *iters = nullptr, *tscratch = nullptr;
    double *logp = nullptr;
    uint32_t *h_iters = nullptr;
    uint8_t *h_ok = nullptr, *h_km = nullptr;
    uint64_t *h_clk = nullptr, *h_seeds = nullptr;  // pinned: the copies stay asynchronous
    double *h_logp = nullptr;
    size_t cap = 0, cap_punct = 0, tscratch_words = 0;
    int f0 = 0, nb = 0;  // the chunk in flight (nb == 0: none)
    qldpc_trials_job *owner = nullptr;  // the job whose results it holds
};

struct DeviceGraph {
    int device = 0;
    int num_cus = 0;
    uint32_t *slot_meta = nullptr;
    int32_t *lane_row0 = nullptr, *lane_head = nullptr, *ell_col = nullptr, *row_deg = nullptr;
    int32_t *wave_rows = nullptr;
    int32_t *lane_nst = nullptr, *lane_epl = nullptr;
    uint32_t *slot_meta_ms = nullptr;                  // V2 min-sum: rows listed by kpos
    uint64_t *vn_mask = nullptr, *vn_mask_ms = nullptr; // V2: [wave][dv_max] slot masks
    uint64_t *vn_exec = nullptr, *vn_exec_ms = nullptr; // V2: [wave][dv_max][slot] lane masks
    uint32_t *slot_meta2 = nullptr, *slot_meta2_ms = nullptr;  // V2 hybrid: stage index per slot
    int32_t *hd_bits = nullptr, *hd_dv = nullptr, *stage_off = nullptr;
    int32_t *row_orig = nullptr;  // V2: layout row -> original row (syndrome index)
    int32_t *part_row0 = nullptr; // V2 split: first layout row of each part
    int32_t *xoff = nullptr;      // V2 split exchange: region starts
    uint16_t *xbit = nullptr, *xbit_ms = nullptr;  // ... chunk-local bit per stage position (CSR / kpos layouts)
    int32_t *iso_bits = nullptr;
    uint32_t *vn_rows = nullptr;  // V2 min-sum bit gather: [n or chunks][2] four u16 layout rows
    uint32_t *vng_bits = nullptr, *vng_meta2 = nullptr;  // hybrid bit gather: bit order, slot positions
    uint32_t *vng_rec = nullptr;  // register-shape bit gather: per slot, the code word's byte offset | shift << 16
    uint64_t *row_sem = nullptr;    // V2 scan: [wave][slot][4] START / END / PARK lane masks (+ pad)
    uint64_t *row_rmask = nullptr;  // V2 scan: [row j][lane] slots of the lane's j-th started row
    int32_t *col_orig = nullptr, *col_lab = nullptr;  // V2 bank relabelling: label -> bit id, bit id -> label
    int32_t *ell_lab = nullptr;     // row-ELL in labels (the claim order reads label-ordered frame codes)
    int32_t *pair_src = nullptr, *pair_col = nullptr;  // v1 occurrence pairing (unsorted adjacency), [k][lane]
    std::mutex mu;     // workspaces (ws), occupancy cache
    std::map<void *, Workspace> ws;
    std::mutex io_mu;  // the host-buffer entry's staging buffers and stream, held copy-in .. copy-out
    HostIO io;
    std::mutex trial_mu;  // qldpc_run_trials' pipeline slots: held while a job enqueues or harvests
    TrialSlot tslot[2];
    int next_slot = 0;    // the slot the next chunk takes (the two alternate)
    int occ[6] = {0, 0, 0, 0, 0, 0};
};

}  // namespace

// Rate-adaptation plan: per position its class (0 key, 1 punctured, 2
// shortened) and source index, replicated on the graph's devices.
struct qldpc_rate_plan {
    struct Dev {
        int device;
        uint8_t *cls;
        int32_t *src;
    };
    int n_punct = 0, n_short = 0;
    std::vector<Dev> devs;
};

namespace {
// Xoshiro256++ (Blackman & Vigna) with Xoshiro-cpp v1.1's seeding (four
// SplitMix64 outputs) — a UniformRandomBitGenerator, so std::shuffle /
// std::uniform_int_distribution consume it exactly as the reference does.
struct Xoshiro256pp {
    using result_type = uint64_t;
    uint64_t s[4];
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    explicit Xoshiro256pp(uint64_t seed) {
        uint64_t x = seed;
        for (auto &v : s) {
            uint64_t z = (x += 0x9e3779b97f4a7c15ull);
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
            v = z ^ (z >> 31);
        }
    }
    static constexpr result_type min() { return 0; }
    static constexpr result_type max() { return ~(uint64_t)0; }
    result_type operator()() {
        const uint64_t r = rotl(s[0] + s[3], 23) + s[0];
        const uint64_t t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
};
}  // namespace

struct qldpc_graph {
    int n = 0, m = 0, E = 0, T = 0, EPL = 0, dv_max = 0, max_dc = 0, variant = 0;
    bool vng = false;                       // V2 min-sum bit gather tables built
    bool vng_h_fit = false;                 // hybrid bit gather's padded edge codes fit LDS (set before planning)
    bool rows_global_ms = false;            // hybrid min-sum: row aggregates (partly) in global scratch
    int rows_lds_ms = 0, rows_lds_waves_ms = 0;  // ... of which the rows of the first waves stay in LDS
    int v2R = 0, v2RG = 0, n_iso = 0;       // V2: register / scratch slots per lane, bits of degree 0
    std::vector<int> wave_rows;             // V2: first layout row of each wave (+ m)
    std::vector<int> row_order;             // V2: layout row -> original row
    std::vector<int> layout_row_ptr;        // V2: row_ptr of the rows in layout order
    int vn_k0 = 0, n_hd = 0;                // V2 hybrid: first staged VN term, bits of degree > vn_k0
    bool paired = false;                    // unsorted adjacency: v1 global-slot kernel with occurrence pairing
    int hd_uniform_dv = 0;                  // > 0: the staged bits are 0..n-1 in order, all of this degree
    int nst_max = 0;                        // V2 SPA scan: most rows started in one lane (row_rmask rows)
    long long stage_doubles = 0;            // V2 hybrid: staged VN terms per frame
    int split_k = 1, split_mrows = 0;       // V2 split: workgroups per frame, rows of the largest part
    int split_cb = 0, split_nc = 0;         // V2 split exchange gather: bits per LDS chunk, chunks per part (0: off)
    int split_pl = REG_TSTRIDE;             // V2 split: a part's lanes (1024: 16 waves; 512: 8 waves, 2 per CU)
    bool kernel_timing = false;             // qldpc_set_kernel_timing
    std::vector<int32_t> col_lab;           // V2 bank relabelling (relabel.cpp): bit id -> label; empty: identity
    long long relabel_stats[4] = {0, 0, 0, 0};  // bank excess before / after, busiest-bank cycles before / after
    std::vector<int> part_row0;             // V2 split: first layout row of each part (+ m)
    std::vector<std::unique_ptr<DeviceGraph>> devs;
};

namespace {

const char *variant_name(int v) {
    switch (v) {
    case VAR_REG_LDS: return "reg_lds";
    case VAR_GLB_LDS: return "glb_lds";
    case VAR_V2: return "v2";
    default: return "glb_glb";
    }
}

// Threads per workgroup: the graph's lanes, or one part's for split frames.
int block_threads(const qldpc_graph &g) {
    return (g.variant == VAR_V2 && g.split_k > 1) ? g.split_pl : g.T;
}

size_t lds_of(const qldpc_graph &g, int alg) {
    if (g.variant == VAR_V2 && g.split_k > 1)
        return lds_bytes_v2(alg, g.n, g.split_mrows, g.split_pl, true, 0, 0, -1, g.split_cb);
    return g.variant == VAR_V2 ? lds_bytes_v2(alg, g.n, g.m, g.T, false, g.v2R, g.v2RG,
                                              (g.rows_global_ms && alg >= 2) ? g.rows_lds_ms : -1)
                               : lds_bytes_for(g.variant, g.n, g.m, g.T);
}

}  // namespace

// The planner's and the launches' A/B knobs (QLDPC_SPLIT_K, QLDPC_VNG, ...)
// are read only under the diagnostic switch QLDPC_DIAG=1: without it the
// product ignores every QLDPC_* tuning variable, so a stray variable in a
// user's environment cannot change the plan the reference's driver gets.
const char *qldpc::qldpc_diag_env(const char *name) {
    const char *d = std::getenv("QLDPC_DIAG");
    if (!d || std::strcmp(d, "1") != 0) return nullptr;
    return std::getenv(name);
}

namespace {

int env_int(const char *name, int dflt) {
    const char *v = qldpc_diag_env(name);
    return (v && *v) ? std::atoi(v) : dflt;
}

int round_up64(long long x) { return (int)(((x + 63) / 64) * 64); }

// Choose (variant, T, EPL).  EPL >= max_dc keeps any row within two lanes;
// lanes past the last edge simply hold no slots.
void plan(qldpc_graph &g) {
    const long long E = g.E;
    const int dcm = std::max(1, g.max_dc);
    // Register-resident messages: at most EPL_REG edges per lane.  (Occurrence
    // pairing reads other lanes' messages: global-slot variants only.)
    if (dcm <= EPL_REG && !g.paired) {
        const int T = std::max(64, round_up64((E + EPL_REG - 1) / EPL_REG));
        const int EPL = std::max((int)((E + T - 1) / T), dcm);
        if (T <= 1024 && EPL <= EPL_REG && lds_bytes_for(VAR_REG_LDS, g.n, g.m, T) <= LDS_LIMIT) {
            g.variant = VAR_REG_LDS;
            g.T = T;
            g.EPL = EPL;
            return;
        }
    }
    // Messages in global scratch: as many lanes as the workgroup allows.
    const int T = (int)std::min<long long>(1024, std::max(64, round_up64((E + 7) / 8)));
    g.T = T;
    g.EPL = std::max((int)((E + T - 1) / T), dcm);
    g.variant = (lds_bytes_for(VAR_GLB_LDS, g.n, g.m, T) <= LDS_LIMIT) ? VAR_GLB_LDS : VAR_GLB_GLB;
}

// V2 plan: rows dealt to W waves in contiguous blocks balanced by edge count,
// each wave's edges dealt EPL_w per lane to its 64 lanes (EPL_w >= max_dc keeps
// a row within two adjacent lanes of ONE wave).  W is the fewest waves whose
// lanes do not need more than max_dc slots (more would only add idle waves
// and barrier cost), capped by the instantiation's workgroup size; R is the
// smallest register-slot instantiation that holds the plan.  QLDPC_V2_WAVES
// forces W.  Returns false when no V2 instantiation fits (v1 is used).
// Deal rows to W waves so that every wave's edge count is at most cap when
// possible: contiguous blocks of rows first (consecutive check ids keep the
// VN phase masks sparse), then swap / move single rows between the heaviest
// and lightest waves.  Returns wave membership lists and the sums.
// With weights wt, wave w's share of the edges is wt[w] / sum(wt) and its cap
// cap * wt[w] (sums compared as sums[w] / wt[w]).
std::vector<std::vector<int>> balance_rows(const int32_t *row_ptr, int m, int W, long long cap,
                                           std::vector<long long> &sums, const std::vector<double> *wt = nullptr) {
    auto deg = [&](int j) { return row_ptr[j + 1] - row_ptr[j]; };
    const long long E = row_ptr[m];
    std::vector<double> cw(W + 1, 0.0);  // cumulative weights
    for (int w = 0; w < W; ++w) cw[w + 1] = cw[w] + (wt ? (*wt)[w] : 1.0);
    auto wof = [&](int w) { return wt ? (*wt)[w] : 1.0; };
    std::vector<std::vector<int>> waves(W);
    sums.assign(W, 0);
    {
        int j = 0;
        for (int w = 0; w < W; ++w) {
            const long long target = wt ? (long long)std::llround((double)E * cw[w + 1] / cw[W]) : E * (w + 1) / W;
            while (j < m && (w == W - 1 || row_ptr[j + 1] <= target ||
                             (row_ptr[j] < target && target - row_ptr[j] > row_ptr[j + 1] - target))) {
                waves[w].push_back(j);
                sums[w] += deg(j);
                ++j;
            }
        }
    }
    // degree -> rows, per wave
    std::vector<std::map<int, std::vector<int>>> by(W);
    for (int w = 0; w < W; ++w)
        for (int j : waves[w]) by[w][deg(j)].push_back(j);
    for (int iter = 0; iter < 100000; ++iter) {
        int H = 0, L = 0;
        for (int w = 1; w < W; ++w) {
            if (sums[w] / wof(w) > sums[H] / wof(H)) H = w;
            if (sums[w] / wof(w) < sums[L] / wof(L)) L = w;
        }
        if (sums[H] <= (long long)(cap * wof(H)) || H == L) break;
        // (weighted: L's normalised load must stay below H's old one)
        const long long gap = wt ? (long long)((double)sums[H] * wof(L) / wof(H)) - sums[L] : sums[H] - sums[L];
        // best transfer d (row of degree dx from H, optionally one of degree dy from L)
        long long best = 0;
        int bx = -1, by_ = -1;
        for (auto &kx : by[H]) {
            if (kx.second.empty()) continue;
            const long long dx = kx.first;
            if (dx < gap && dx > best) best = dx, bx = kx.first, by_ = -1;  // move
            for (auto &ky : by[L]) {
                if (ky.second.empty()) continue;
                const long long d = dx - ky.first;
                if (d > 0 && d < gap && d > best) best = d, bx = kx.first, by_ = ky.first;
            }
        }
        if (best == 0) break;
        // never overshoot: the new max of the pair must drop
        const int x = by[H][bx].back();
        by[H][bx].pop_back();
        by[L][bx].push_back(x);
        sums[H] -= bx;
        sums[L] += bx;
        if (by_ >= 0) {
            const int y = by[L][by_].back();
            by[L][by_].pop_back();
            by[H][by_].push_back(y);
            sums[L] -= by_;
            sums[H] += by_;
        }
    }
    for (int w = 0; w < W; ++w) {
        waves[w].clear();
        for (auto &kv : by[w]) waves[w].insert(waves[w].end(), kv.second.begin(), kv.second.end());
        std::sort(waves[w].begin(), waves[w].end());
    }
    return waves;
}

// V2 plan: rows dealt to W waves (balanced by edge count, rows relabelled so
// each wave holds a contiguous block of layout rows), each wave's edges dealt
// EPL_w per lane to its 64 lanes (EPL_w >= max_dc keeps a row within two
// adjacent lanes of ONE wave).  W is the fewest waves whose lanes do not need
// more than max_dc slots (more would only add idle waves and barrier cost),
// capped by the instantiation's workgroup size; the shape is the smallest
// slot count that holds the plan.  QLDPC_V2_WAVES forces W.  Returns false when
// no V2 instantiation fits (v1 is used).
bool plan_v2(qldpc_graph &g, const int32_t *row_ptr) {
    // head <= 31 (tail parity in a 32-bit mask), dummy column id n < 2^20
    if (g.max_dc <= 0 || g.max_dc > 32 || g.n + 1 > (int)META_COL_MASK || g.n > V2_CODES_CAP) return false;
    for (int j = 0; j < g.m; ++j)
        if (row_ptr[j + 1] == row_ptr[j]) return false;  // empty rows: v1 checks them by row-ELL
    const long long E = g.E;
    const int forced = env_int("QLDPC_V2_WAVES", 0);
    const int shapes[4][2] = {{V2_R_TIGHT, 0}, {V2_R_SMALL, 0}, {V2_R_MID, 0}, {V2_R_SMALL, V2_RG_HYBRID}};
    // register shapes (RG == 0) scan from 64-bit lane-mask rows of at most 63
    // slots (row_rmask bit 63 marks a row continuing into the next lane)
    static_assert(V2_R_TIGHT <= 63 && V2_R_SMALL <= 63 && V2_R_MID <= 63, "register shape beyond the scan's masks");
    for (const auto &sh : shapes) {
        const int R = sh[0] + sh[1];  // slots per lane
        const int wmax = v2_threads_for(sh[0]) / 64;
        int W = forced > 0 ? forced : (int)std::min<long long>(wmax, (E + 64LL * g.max_dc - 1) / (64LL * g.max_dc));
        W = std::max(1, W);
        if (W > wmax) continue;
        // min-sum row aggregates (16 B/row) must fit beside the totals; on the
        // hybrid shape they may live in global scratch instead when the bit
        // gather applies (then only the SPA image, 8 B/row, must fit)
        bool rows_global = false;
        // (the shape's own layout: the mask-driven scan's syndrome words exist
        // on the register shapes only)
        if (lds_bytes_v2(2, g.n, g.m, W * 64, false, sh[0], sh[1]) > LDS_LIMIT) {
            if (sh[1] == 0 || !g.vng_h_fit || g.m >= 0xFFFF ||
                lds_bytes_v2(0, g.n, g.m, W * 64, false, sh[0], sh[1]) > LDS_LIMIT ||
                lds_bytes_v2(2, g.n, g.m, W * 64, false, sh[0], sh[1], 0) > LDS_LIMIT)
                continue;
            rows_global = true;
        }
        const long long cap = 64LL * std::max<long long>((E + 64LL * W - 1) / (64LL * W), g.max_dc);
        std::vector<long long> sums;
        std::vector<int> order, rb(W + 1, 0), nrp(g.m + 1, 0);
        int wl = W, epl = 0;
        // Deal the rows with the waves past the first wl given `share` of a
        // wave's edges; false when some lane would exceed the shape.
        auto deal = [&](double share) -> bool {
            std::vector<double> wt(W, 1.0);
            wl = W;
            for (int pass = 0; pass < 6; ++pass) {
                const bool weighted = share != 1.0 && pass > 0;
                const long long capw = weighted ? 64LL * std::max<long long>(
                    (long long)std::ceil((double)E / (wl + (W - wl) * share) / 64.0), g.max_dc) : cap;
                const auto waves = balance_rows(row_ptr, g.m, W, capw, sums, weighted ? &wt : nullptr);
                order.clear();
                for (int w = 0; w < W; ++w) {
                    order.insert(order.end(), waves[w].begin(), waves[w].end());
                    rb[w + 1] = (int)order.size();
                }
                for (int jr = 0; jr < g.m; ++jr)
                    nrp[jr + 1] = nrp[jr] + (row_ptr[order[jr] + 1] - row_ptr[order[jr]]);
                if (!rows_global) break;
                int wn = env_int("QLDPC_ROWS_LDS", 1) ? W : 0;
                while (wn > 0 && lds_bytes_v2(2, g.n, g.m, W * 64, false, sh[0], sh[1], rb[wn]) > LDS_LIMIT) --wn;
                const bool agree = share == 1.0 || (pass > 0 && wn == wl);
                wl = wn;
                if (agree) break;
                for (int w = 0; w < W; ++w) wt[w] = w < wl ? 1.0 : share;
            }
            epl = 0;
            for (int w = 0; w < W; ++w) {
                const long long ew = nrp[rb[w + 1]] - nrp[rb[w]];
                if (ew == 0) continue;
                const int e = std::max<int>((int)((ew + 63) / 64), g.max_dc);
                if (e > R) return false;
                epl = std::max(epl, e);
                // rows started per lane must fit the 32-bit syndrome mask
                for (long long l = 0; l < 64; ++l) {
                    const long long e0 = nrp[rb[w]] + l * e, e1 = std::min<long long>(e0 + e, nrp[rb[w + 1]]);
                    int starts = 0;
                    for (int jr = rb[w]; jr < rb[w + 1]; ++jr)
                        if (nrp[jr] >= e0 && nrp[jr] < e1) ++starts;
                    if (starts > 32) return false;
                }
            }
            return true;
        };
        // Rows partly in global scratch: the waves whose rows stay in LDS are
        // the leading wl (as many as fit); the others write their rows to L2
        // in the scan and read them back (the gather, and the copy their
        // message pass reads).  Those get a smaller share of a wave's edges
        // so the phase barriers do not wait on them (R=0.5 code: 80% is 4%
        // faster than an even deal and 5% faster than 65%, tools/env_ab.sh)
        // — the smallest share from QLDPC_RGLB_SHARE (percent) up whose deal
        // fits the shape.  wl depends on the deal, so each deal is redone
        // until they agree.
        bool ok = false;
        const int share0 = rows_global ? std::min(100, std::max(10, env_int("QLDPC_RGLB_SHARE", 80))) : 100;
        for (int sp = share0; sp <= 100 && !ok; sp += 5) ok = deal(sp / 100.0);
        if (!ok) continue;
        g.variant = VAR_V2;
        g.v2R = sh[0];
        g.v2RG = sh[1];
        g.rows_global_ms = rows_global;
        g.rows_lds_ms = g.m;
        g.rows_lds_waves_ms = W;
        if (rows_global) {
            // the rows of the leading wl waves stay in LDS beside the totals
            // (QLDPC_ROWS_LDS=0: none, A/B)
            g.rows_lds_waves_ms = wl;
            g.rows_lds_ms = rb[wl];
        }
        g.T = W * 64;
        g.EPL = epl;
        g.wave_rows = rb;
        g.row_order = order;
        g.layout_row_ptr = nrp;
        return true;
    }
    return false;
}

// V2 split plan, for codes whose frame does not fit one CU (totals beyond LDS
// or more edges than 16 waves x 64 lanes x 40 slots): K parts of WR waves
// each (one workgroup per part), rows dealt to the WR K waves as in plan_v2
// (contiguous balanced blocks).  Totals go to global memory.  Parts are 16
// waves (one per CU), or 8 waves (two per CU, half the LDS each) when that
// lets more frames run at once on an XCD's 32 CUs: a frame's time per
// iteration is set by latency, not by its part count (C4 (ii), n = 102400,
// dv = 4: K = 11, 12 and 16 parts of 16 waves decode in the same 24.0-24.1 ms,
// two frames per XCD each — 32 = 2 x 11 + 10 leaves 10 CUs waiting; with
// 8-wave parts K = 21 runs three per XCD).  The graph's per-part arrays keep
// a stride of 16 waves / REG_TSTRIDE lanes either way (8-wave parts leave
// waves 8..15 of each part empty), so part r = waves [16r, 16r + 16).
// QLDPC_SPLIT=0 disables it (v1 is used); QLDPC_SPLIT_K / QLDPC_SPLIT_WP force
// the part count / size.
bool plan_v2_split(qldpc_graph &g, const int32_t *row_ptr, const int32_t *col_idx) {
    if (env_int("QLDPC_SPLIT", 1) == 0) return false;
    if (g.max_dc <= 0 || g.max_dc > 32 || g.n + 1 > (int)META_COL_MASK) return false;
    for (int j = 0; j < g.m; ++j)
        if (row_ptr[j + 1] == row_ptr[j]) return false;
    const long long E = g.E;
    const int WP = REG_TSTRIDE / 64;  // waves per part in the graph's arrays
    // One attempt: K parts of WR waves, V2_R_SPLIT slots per lane in VGPRs /
    // LDS plus RG in per-workgroup global scratch.
    auto attempt = [&](int K, int RG, int WR) -> bool {
        const int R = V2_R_SPLIT + RG;
        const int PL = WR * 64;                                  // the part's lanes (threads)
        const size_t LIM = (size_t)LDS_LIMIT * WR / WP;           // its LDS: 1 or 2 parts per CU
        const int W = WP * K, Wr = WR * K;
        const long long cap = 64LL * std::max<long long>((E + 64LL * Wr - 1) / (64LL * Wr), g.max_dc);
        if (cap > 64LL * R) return false;
        std::vector<long long> sums;
        const auto waves = balance_rows(row_ptr, g.m, Wr, cap, sums);
        std::vector<int> order, rb(W + 1, 0), nrp(g.m + 1, 0);
        for (int w = 0; w < W; ++w) {  // wave w = part w / WP, its (w % WP)-th wave (empty past WR)
            if (w % WP < WR) {
                const auto &wr = waves[(w / WP) * WR + w % WP];
                order.insert(order.end(), wr.begin(), wr.end());
            }
            rb[w + 1] = (int)order.size();
        }
        if ((int)order.size() != g.m) return false;
        for (int j = 0; j < g.m; ++j) nrp[j + 1] = nrp[j] + (row_ptr[order[j] + 1] - row_ptr[order[j]]);
        int epl = 0;
        bool ok = true;
        for (int w = 0; w < W && ok; ++w) {
            const long long ew = nrp[rb[w + 1]] - nrp[rb[w]];
            if (ew == 0) continue;
            const int e = std::max<int>((int)((ew + 63) / 64), g.max_dc);
            ok = e <= R;
            epl = std::max(epl, e);
            for (long long l = 0; l < 64 && ok; ++l) {
                const long long e0 = nrp[rb[w]] + l * e, e1 = std::min<long long>(e0 + e, nrp[rb[w + 1]]);
                int starts = 0;
                for (int j = rb[w]; j < rb[w + 1]; ++j)
                    if (nrp[j] >= e0 && nrp[j] < e1) ++starts;
                ok = starts <= 32;
            }
        }
        if (!ok) return false;
        std::vector<int> prow(K + 1);
        int mrows = 0;
        for (int r = 0; r <= K; ++r) prow[r] = rb[std::min(W, r * WP)];
        for (int r = 0; r < K; ++r) mrows = std::max(mrows, prow[r + 1] - prow[r]);
        if (lds_bytes_v2(2, g.n, mrows, PL, true, 0, 0, -1, 0) > LIM ||
            lds_bytes_v2(0, g.n, mrows, PL, true, 0, 0, -1, 0) > LIM)
            return false;
        // Exchange gather (DecodeArgs::xoff): the largest LDS chunk of a part's
        // bits every algorithm's layout holds (SPA keeps its LDS message slots
        // when they fit without it), split evenly; QLDPC_SPLIT_X=0: the
        // term-major stage (A/B).
        int cb = 0, nc = 0;
        if (env_int("QLDPC_SPLIT_X", 1)) {
            const int own = (g.n + K - 1) / K;
            const bool rl0 = v2_split_rl_fits(g.n, mrows, 0, PL);
            auto fits = [&](int c) {
                return lds_bytes_v2(2, g.n, mrows, PL, true, 0, 0, -1, c) <= LIM &&
                       lds_bytes_v2(0, g.n, mrows, PL, true, 0, 0, -1, c) <= LIM &&
                       (!rl0 || v2_split_rl_fits(g.n, mrows, c, PL));
            };
            int lo = 0, hi = std::min(own, 0xFFFF);
            while (lo < hi) {
                const int mid = (lo + hi + 1) / 2;
                if (fits(mid)) lo = mid;
                else hi = mid - 1;
            }
            if (lo >= 256) {
                nc = (own + lo - 1) / lo;
                cb = (own + nc - 1) / nc;
            }
        }
        g.variant = VAR_V2;
        g.v2R = V2_R_SPLIT;
        g.v2RG = RG;
        g.T = W * 64;
        g.EPL = epl;
        g.wave_rows = rb;
        g.row_order = order;
        g.layout_row_ptr = nrp;
        g.split_k = K;
        g.split_mrows = mrows;
        g.part_row0 = prow;
        g.split_cb = cb;
        g.split_nc = nc;
        g.split_pl = PL;
        return true;
    };
    // The smallest feasible K for each part size, then the size that runs more
    // frames per XCD at once (32 CUs: 32 parts of 16 waves or 64 of 8; ties:
    // 8 waves — C4 stand-in, 4 frames per XCD either way: 15 x 8 waves decode
    // as fast as 8 x 16 and the step runs 4% faster, profiles/r05/c4_wp.txt).  (K need not divide an XCD's parts:
    // groups form in claim order and a workgroup joins the next group whenever
    // it finishes a frame.)
    //
    // Scratch message slots (RG = V2_RG_SPLIT, round 6): 52 slots per lane
    // instead of 40 cut the parts per frame by ~1/4, at a cost — each part's
    // passes hold ~1.3x the edges and the scratch slots travel through L2.
    // Four plan families (part size x slot budget), each at its smallest K.
    // Per slot budget the family with the most frames per XCD wins, ties in
    // the measured order (profiles/r06/split_plans/, 2-stream bench, two split
    // launches in flight): without scratch slots 8-wave parts (two per CU),
    // then 16-wave; with them 16-wave parts (one per CU: half the parts per
    // frame), then 8-wave.  The scratch-slot plan is taken when it runs at
    // least 4/3 the frames per XCD of the plan without: C4 (ii) 8w/0 21 parts
    // (3 frames per XCD) 0.59 Gbit/s, 16w/12 8 parts (4) 0.68 <- taken (8w/12
    // 16 parts: 0.62); the stand-in 8w/0 15 parts (4) 0.451 <- kept, 16w/12 6
    // parts (5) 0.457 at 1.4x the HBM+MALL traffic and a slower decode alone
    // (16w/0 8 parts: 0.436, 8w/12 12 parts: 0.437).  QLDPC_SPLIT_WP (8 / 16)
    // and QLDPC_SPLIT_SCRATCH (0 / 1), diagnostic, restrict the families.
    const int kforce = env_int("QLDPC_SPLIT_K", 0);
    const int wforce = env_int("QLDPC_SPLIT_WP", 0);
    const int sforce = env_int("QLDPC_SPLIT_SCRATCH", -1);
    if (wforce && wforce != 16 && wforce != 8) return false;
    auto smallest_k = [&](int WR, int RG) -> int {
        const long long cap_part = (long long)WR * 64 * (V2_R_SPLIT + RG);
        const int kmin = (int)std::max<long long>(2, (E + cap_part - 1) / cap_part);
        if (kforce) return (kforce >= kmin && kforce <= 32 && attempt(kforce, RG, WR)) ? kforce : 0;
        for (int K = kmin; K <= 32; ++K)
            if (attempt(K, RG, WR)) return K;
        return 0;
    };
    struct Plan {
        int K = 0, WR = 0, RG = 0, f = 0;
    };
    auto best_of = [&](int RG, int first_wr) -> Plan {  // the better part size for one slot budget
        Plan b;
        for (int WR : {first_wr, 24 - first_wr}) {
            if (wforce && WR != wforce) continue;
            const int K = smallest_k(WR, RG);
            const int f = K ? (WR == 8 ? 64 : 32) / K : 0;  // frames per XCD (32 CUs)
            if (f > b.f) b = {K, WR, RG, f};                 // (ties keep the first size)
        }
        return b;
    };
    const Plan p0 = sforce == 1 ? Plan{} : best_of(0, 8);
    const Plan ps = sforce == 0 ? Plan{} : best_of(V2_RG_SPLIT, 16);
    const Plan pick = (ps.K && (!p0.K || 3 * ps.f >= 4 * p0.f)) ? ps : p0;
    if (!pick.K) return false;
    return attempt(pick.K, pick.RG, pick.WR);  // (the last attempt sets the plan)
}

template <typename T>
int upload(T **dst, const std::vector<T> &src) {
    const size_t bytes = std::max<size_t>(1, src.size()) * sizeof(T);
    HIP_TRY(hipMalloc(dst, bytes));
    if (!src.empty()) HIP_TRY(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return QLDPC_OK;
}

// Labellings already searched in this process (relabel.cpp takes ~0.5 s on a
// 10k code; tests and drivers create graphs of one H many times).  Keyed by a
// hash of everything the search reads, verified by a full compare on a hit.
struct RelabelMemo {
    std::vector<int32_t> key;  // n, m, waves, mode, iters, row_ptr..., col_idx...
    std::vector<int32_t> lab;
    long long stats[4];
};
std::mutex g_relabel_mu;
std::vector<RelabelMemo> g_relabel_memo;  // most recent last, at most 8

// host_only: plan and relabel without any device (introspection; the graph
// has no devices and cannot decode).
// bit_nodes (col_ptr / row_idx, the reference's H_matrix::bit_nodes in its
// own order): NULL means the ascending transpose of check_nodes.
int build_graph(int32_t n, int32_t m, const int32_t *row_ptr, const int32_t *col_idx, int32_t device_mask,
                qldpc_graph **out, bool host_only = false, const std::vector<int> *device_list = nullptr,
                const int32_t *col_ptr = nullptr, const int32_t *row_idx = nullptr) {
    if (!out) return fail(QLDPC_EINVAL, "out is NULL");
    *out = nullptr;
    if (n <= 0 || m < 0 || !row_ptr || (!col_idx && row_ptr[m] > 0))
        return fail(QLDPC_EINVAL, "invalid graph dimensions or NULL arrays");
    if (n > MAX_N) return fail(QLDPC_EUNSUP, "n exceeds 2^20 bit nodes");
    if (row_ptr[0] != 0) return fail(QLDPC_EINVAL, "row_ptr[0] must be 0");
    for (int j = 0; j < m; ++j)
        if (row_ptr[j + 1] < row_ptr[j]) return fail(QLDPC_EINVAL, "row_ptr must be non-decreasing");
    const int E = row_ptr[m];
    if (E <= 0) return fail(QLDPC_EINVAL, "graph has no edges");

    auto g = std::make_unique<qldpc_graph>();
    g->n = n;
    g->m = m;
    g->E = E;
    std::vector<int> dv(n, 0);
    bool rows_sorted = true;
    for (int j = 0; j < m; ++j) {
        g->max_dc = std::max(g->max_dc, row_ptr[j + 1] - row_ptr[j]);
        for (int e = row_ptr[j]; e < row_ptr[j + 1]; ++e) {
            const int c = col_idx[e];
            if (c < 0 || c >= n) return fail(QLDPC_EINVAL, "col_idx entry out of range [0, n)");
            if (e > row_ptr[j] && col_idx[e - 1] >= c) rows_sorted = false;
            ++dv[c];
        }
    }
    // The reference pairs a check's k-th input with the k-th time the VN loop
    // visits that check (bit_pos_idx, src/qkd_ldpc_algorithm.cpp:116-118) and
    // a bit's k-th message with the k-th check that reached it (check_pos_idx,
    // :67-69).  With ascending check_nodes rows and bit_nodes their ascending
    // transpose both pairings are the edge itself; otherwise an edge's b2c is
    // total - c2b of the edge the counters pair it with (occurrence pairing).
    if (!rows_sorted) {
        for (int j = 0; j < m; ++j) {  // (a bit listed twice in one check is not supported)
            std::vector<int32_t> r(col_idx + row_ptr[j], col_idx + row_ptr[j + 1]);
            std::sort(r.begin(), r.end());
            if (std::adjacent_find(r.begin(), r.end()) != r.end())
                return fail(QLDPC_EUNSUP, "a check node lists the same bit twice");
        }
    }
    bool cols_transpose = true;
    if (col_ptr && row_idx) {
        if (col_ptr[0] != 0 || col_ptr[n] != row_ptr[m])
            return fail(QLDPC_EUNSUP, "bit_nodes and check_nodes hold different edge counts");
        std::vector<int> cnt(m, 0);
        for (int i = 0; i < n; ++i) {
            if (col_ptr[i + 1] < col_ptr[i]) return fail(QLDPC_EINVAL, "col_ptr must be non-decreasing");
            if (col_ptr[i + 1] - col_ptr[i] != dv[i])
                return fail(QLDPC_EUNSUP, "bit_nodes and check_nodes disagree on a bit's degree");
            for (int e = col_ptr[i]; e < col_ptr[i + 1]; ++e) {
                const int j = row_idx[e];
                if (j < 0 || j >= m) return fail(QLDPC_EINVAL, "row_idx entry out of range [0, m)");
                ++cnt[j];
            }
        }
        for (int j = 0; j < m; ++j)
            if (cnt[j] != row_ptr[j + 1] - row_ptr[j])
                return fail(QLDPC_EUNSUP, "bit_nodes and check_nodes disagree on a check's degree");
        // bit_nodes[c] must list the checks holding c in ascending order (the
        // order the check-node loop reaches c in) for the identity pairing
        std::vector<int> fill(n, 0);
        for (int j = 0; j < m && cols_transpose; ++j)
            for (int e = row_ptr[j]; e < row_ptr[j + 1]; ++e) {
                const int c = col_idx[e];
                if (row_idx[col_ptr[c] + fill[c]++] != j) {
                    cols_transpose = false;
                    break;
                }
            }
    }
    g->paired = !(rows_sorted && cols_transpose);
    for (int i = 0; i < n; ++i) g->dv_max = std::max(g->dv_max, dv[i]);
    {
        long long chunks = 0;
        for (int i = 0; i < n; ++i) chunks += (dv[i] + 3) / 4;
        g->vng_h_fit = chunks + V2_VNG_DUMMY_CHUNKS <= V2_CODES_CAP && g->dv_max < 256;
    }
    if (g->dv_max >= MAX_DV) return fail(QLDPC_EUNSUP, "a bit node has degree >= 511");
    // QLDPC_VARIANT=v1 keeps the first-generation planner (comparison / tests).
    const char *want = qldpc_diag_env("QLDPC_VARIANT");
    const bool v1_only = want && std::strcmp(want, "v1") == 0;
    if (g->paired && want && std::strcmp(want, "v2") == 0)
        return fail(QLDPC_EUNSUP, "QLDPC_VARIANT=v2 but the adjacency needs occurrence pairing (v1)");
    if (v1_only || g->paired || (!plan_v2(*g, row_ptr) && !plan_v2_split(*g, row_ptr, col_idx))) plan(*g);
    if (want && std::strcmp(want, "v2") == 0 && g->variant != VAR_V2)
        return fail(QLDPC_EUNSUP, "QLDPC_VARIANT=v2 but no V2 instantiation holds this graph");
    const int T = g->T, EPL = g->EPL;
    std::vector<int32_t> iso;
    for (int i = 0; i < n; ++i)
        if (dv[i] == 0) iso.push_back(i);
    g->n_iso = (int)iso.size();

    // Lane partition metadata.
    std::vector<int> row_of(E), kpos(E), seen(n, 0);
    for (int j = 0; j < m; ++j)
        for (int e = row_ptr[j]; e < row_ptr[j + 1]; ++e) {
            row_of[e] = j;
            kpos[e] = seen[col_idx[e]]++;
        }
    // uint4 groups per lane, group-major [g][lane][4]; the register variants
    // have a fixed group count at lane stride REG_TSTRIDE.
    const bool v2 = g->variant == VAR_V2;
    const bool reg = g->variant == VAR_REG_LDS || v2;
    const int G4 = v2 ? (g->v2R + g->v2RG) / 4 : (reg ? EPL_REG / 4 : (EPL + 3) / 4);
    const int TS = reg ? REG_TSTRIDE : T;
    const int NPARTS = (T + TS - 1) / TS;  // V2 split: parts of TS lanes, each its own [G4][TS][4] block
    auto midx = [&](int l, int k) -> size_t {
        return ((size_t)((l / TS) * G4 + k / 4) * TS + (size_t)(l % TS)) * 4 + (size_t)(k % 4);
    };
    std::vector<uint32_t> meta((size_t)G4 * TS * 4 * NPARTS, 0);
    std::vector<int32_t> lrow0(T, v2 ? 0 : -1), lhead(T, 0), lnst(T, 0), lepl(T, EPL);
    // Lane l holds edges [e_begin, e_end) of its wave (v1: one "wave" of T lanes).
    // V2 metadata differs in three ways: the END of a lane's tail (a row begun
    // in the lane before) is cleared — the kernel finishes split rows after a
    // shuffle; slots past the lane's edges up to the group count are dummy
    // edges (column n, kpos META_KPOS_MASK, no flags), so every lane of a wave
    // runs the same slots; lanes count the rows they start (lane_nst).
    const uint32_t DUMMY = (uint32_t)n | (META_KPOS_MASK << META_KPOS_SHIFT);
    const int W = v2 ? T / 64 : 1;
    // V2 min-sum metadata lists each row's edges by kpos: the min-sum row
    // aggregate and parity are order-free, and grouping a
    // row's k-th bit edges lets the VN phase masks skip more slots.  SPA keeps
    // CSR order (its row product is sequential, :57-62).
    // Layout order: V2 relabels rows (plan_v2 balances waves); lrp / lrow /
    // ledge give, per position of the layout's row-major edge list, its row
    // and its original CSR edge.  v1 keeps the original order.
    std::vector<int> lrp(row_ptr, row_ptr + m + 1), lrow(row_of), ledge(E), perm(E);
    for (int e = 0; e < E; ++e) ledge[e] = e;
    if (v2) {
        lrp = g->layout_row_ptr;
        for (int j = 0; j < m; ++j) {
            const int r = g->row_order[j];
            for (int t = 0; t < row_ptr[r + 1] - row_ptr[r]; ++t) {
                lrow[lrp[j] + t] = j;
                ledge[lrp[j] + t] = row_ptr[r] + t;
            }
        }
    }
    // Bank-aware relabelling of bit ids (relabel.cpp), one-workgroup register
    // shapes: the (wave, slot, half) groups of both slot layouts (CSR order for
    // the SPA family, kpos order for min-sum) read total[label] with distinct
    // banks, and the min-sum bit gather's code-word ORs (dv <= 4) hit distinct
    // banks too.  The metadata, vn_rows and vng_rec then carry labels; the frame
    // codes are written in label order and the decoder maps its outputs back.
    // QLDPC_RELABEL=0: identity (A/B).
    std::vector<int32_t> col_r;
    const int32_t *colL = col_idx;  // the metadata's bit ids
    const int relabel_mode = env_int("QLDPC_RELABEL", 1);  // (A/B: 2 CSR layout only, 3 kpos layout only)
    if (v2 && g->split_k <= 1 && g->v2RG == 0 && relabel_mode != 0) {
        const bool word = v2_vng_ok(2, g->v2R, g->v2RG, g->split_k, g->dv_max, m);
        std::vector<RelabelGroup> groups;
        for (int sorted = 0; sorted < 2; ++sorted) {
            if ((relabel_mode == 2 && sorted) || (relabel_mode == 3 && !sorted)) continue;
            std::vector<int> pm(ledge);
            if (sorted)
                for (int j = 0; j < m; ++j)
                    std::stable_sort(pm.begin() + lrp[j], pm.begin() + lrp[j + 1],
                                     [&](int x, int y) { return kpos[x] < kpos[y]; });
            for (int w = 0; w < T / 64; ++w) {
                const long long wb = lrp[g->wave_rows[w]], we = lrp[g->wave_rows[w + 1]];
                const int epl_w = std::max<int>((int)((we - wb + 63) / 64), g->max_dc);
                if (we == wb) continue;
                for (int k = 0; k < epl_w; ++k)
                    for (int h = 0; h < 2; ++h) {
                        RelabelGroup grp;
                        for (int li = 32 * h; li < 32 * h + 32; ++li) {
                            const long long e = wb + (long long)li * epl_w + k;
                            if (e < we) {
                                const int ed = pm[e];
                                grp.members.push_back({col_idx[ed], 0, (uint8_t)(1 | ((sorted && word && kpos[ed] < 4) ? 2 : 0))});
                            } else {
                                grp.members.push_back({-1, n % 128, 1});  // dummy slot: column n
                            }
                        }
                        groups.push_back(std::move(grp));
                    }
            }
        }
        const int iters = env_int("QLDPC_RELABEL_ITERS", 16);  // search moves per edge
        std::vector<int32_t> key = {n, m, T / 64, relabel_mode, iters};
        key.insert(key.end(), row_ptr, row_ptr + m + 1);
        key.insert(key.end(), col_idx, col_idx + E);
        {
            std::lock_guard<std::mutex> lk(g_relabel_mu);
            for (const auto &me : g_relabel_memo)
                if (me.key == key) {
                    g->col_lab = me.lab;
                    std::copy(me.stats, me.stats + 4, g->relabel_stats);
                    break;
                }
        }
        if (g->col_lab.empty()) {
            RelabelStats st;
            g->col_lab = bank_relabel(n, groups, 0x5eed0ba4c5ull, (long long)iters * E, &st);
            g->relabel_stats[0] = st.excess_before;
            g->relabel_stats[1] = st.excess_after;
            g->relabel_stats[2] = st.cycles_before;
            g->relabel_stats[3] = st.cycles_after;
            std::lock_guard<std::mutex> lk(g_relabel_mu);
            if (g_relabel_memo.size() >= 8) g_relabel_memo.erase(g_relabel_memo.begin());
            g_relabel_memo.push_back({std::move(key), g->col_lab, {g->relabel_stats[0], g->relabel_stats[1],
                                                                    g->relabel_stats[2], g->relabel_stats[3]}});
        }
        col_r.resize(E);
        for (int e = 0; e < E; ++e) col_r[e] = g->col_lab[col_idx[e]];
        colL = col_r.data();
    }
    // Hybrid shape: VN terms kk >= vn_k0 go through a per-frame stage, laid out
    // term-major over the bits of degree > kk, bits ordered by degree
    // (descending) so each term's bits are a prefix: stage[off[kk] + rank[b]].
    g->vn_k0 = g->dv_max;
    std::vector<int32_t> hd_bits, hd_dv, stage_off(std::max(1, g->dv_max), 0), rank(n, -1);
    // (split frames: every term goes through the stage, and the gather pass
    // adds them to the channel LLR in order: the message pass stores only)
    if (v2 && ((g->v2RG > 0 && g->dv_max > 4) || (g->split_k > 1 && g->dv_max >= 1))) {
        g->vn_k0 = g->split_k > 1 ? 0 : 4;
        for (int i = 0; i < n; ++i)
            if (dv[i] > g->vn_k0) hd_bits.push_back(i);
        std::stable_sort(hd_bits.begin(), hd_bits.end(), [&](int x, int y) { return dv[x] > dv[y]; });
        for (size_t i = 0; i < hd_bits.size(); ++i) {
            rank[hd_bits[i]] = (int)i;
            hd_dv.push_back(dv[hd_bits[i]]);
        }
        long long off = 0;
        for (int kk = g->vn_k0; kk < g->dv_max; ++kk) {
            stage_off[kk] = (int32_t)off;
            for (int d : hd_dv) off += (d > kk) ? 1 : 0;
        }
        g->stage_doubles = off;
    }
    g->n_hd = (int)hd_bits.size();
    if (g->n_hd == n && n > 0) {
        bool uni = true;
        for (int i = 0; i < n && uni; ++i) uni = hd_bits[i] == i && hd_dv[i] == hd_dv[0];
        g->hd_uniform_dv = (uni && env_int("QLDPC_HD_TABLES", 0) == 0) ? hd_dv[0] : 0;  // (env: A/B)
    }
    const int S4 = G4 * 4;  // V2 slots per lane (register + scratch)
    // Min-sum bit gather (VNG).  Register shape, dv <= 4: per bit, the layout
    // rows of its kpos-th edge (u16 each, 0xFFFF past its degree).  Hybrid
    // shape: a bit's edges padded to chunks of four (position P0[b] + kpos),
    // rows per chunk (padding: row 0), each slot's position (vng_meta2; dummy
    // slots: a scratch chunk per lane past the last), bits in degree order.
    std::vector<uint32_t> vn_rows, vng_bits, vng_meta2;
    long long vng_chunks = 0;
    std::vector<long long> P0(v2 ? n : 0, 0);
    if (v2 && v2_vng_ok(2, g->v2R, g->v2RG, g->split_k, g->dv_max, m)) {
        std::vector<int> lrow_of(m, 0);
        for (int j = 0; j < m; ++j) lrow_of[g->row_order[j]] = j;
        if (g->v2RG == 0) {
            vn_rows.assign((size_t)2 * n, 0xFFFFFFFFu);
            for (int r = 0; r < m; ++r)
                for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e) {
                    uint32_t &w = vn_rows[(size_t)2 * colL[e] + (kpos[e] >> 1)];
                    const int sh = 16 * (kpos[e] & 1);
                    w = (w & ~(0xFFFFu << sh)) | ((uint32_t)lrow_of[r] << sh);
                }
        } else {
            for (int b = 0; b < n; ++b) {
                P0[b] = vng_chunks * 4;
                vng_chunks += (dv[b] + 3) / 4;
            }
            if (vng_chunks + V2_VNG_DUMMY_CHUNKS <= V2_CODES_CAP && g->dv_max < 256) {
                vn_rows.assign((size_t)2 * vng_chunks, 0u);
                for (int r = 0; r < m; ++r)
                    for (int e = row_ptr[r]; e < row_ptr[r + 1]; ++e) {
                        const long long P = P0[col_idx[e]] + kpos[e];
                        vn_rows[(size_t)(P >> 1)] |= (uint32_t)lrow_of[r] << (16 * (P & 1));
                    }
                std::vector<int> ord(n);
                for (int b = 0; b < n; ++b) ord[b] = b;
                std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return dv[x] > dv[y]; });
                // Thread t gathers positions t, t + T, ...: wave w's lanes take
                // the 64-bit groups at j T + 64 w.  Groups of 64 consecutive
                // bits in degree order (similar chunk counts: no lane idles
                // long) are dealt longest-first to the wave with the least
                // work so far, so the gather's barrier does not wait on the
                // waves that drew the high-degree bits (QLDPC_VNG_DEAL=0: in
                // order).  Only full rounds are dealt; the rest stays in order.
                const int TW = g->T / 64, rounds = n / g->T;
                if (env_int("QLDPC_VNG_DEAL", 1) && TW > 1 && rounds > 1) {
                    const int ng = rounds * TW;
                    std::vector<long long> load(TW, 0);
                    std::vector<int> used(TW, 0), dst(ng);
                    for (int gi = 0; gi < ng; ++gi) {  // groups come longest first
                        const long long cost = (dv[ord[(size_t)gi * 64]] + 3) / 4;
                        int best = -1;
                        for (int w = 0; w < TW; ++w)
                            if (used[w] < rounds && (best < 0 || load[w] < load[best])) best = w;
                        dst[gi] = used[best]++ * g->T + 64 * best;
                        load[best] += cost;
                    }
                    std::vector<int> dealt(ord);
                    for (int gi = 0; gi < ng; ++gi)
                        for (int l = 0; l < 64; ++l) dealt[dst[gi] + l] = ord[(size_t)gi * 64 + l];
                    ord.swap(dealt);
                }
                vng_bits.resize((size_t)2 * n);
                for (int i = 0; i < n; ++i) {
                    vng_bits[2 * i] = (uint32_t)ord[i];
                    vng_bits[2 * i + 1] = (uint32_t)(P0[ord[i]] / 4) | ((uint32_t)dv[ord[i]] << 24);
                }
                vng_meta2.assign((size_t)G4 * TS * 4 * NPARTS, 0);
            }
        }
    }
    const bool vng_h = !vng_meta2.empty();
    // Register-shape bit gather: per slot where the message pass ORs the
    // edge's two bits — the byte offset of the bit's code word and the
    // shift of its kpos-th bit pair (8 (col & 3) + 2 kpos).
    std::vector<uint32_t> vng_rec;
    if (v2 && !vn_rows.empty() && g->v2RG == 0) vng_rec.assign((size_t)G4 * TS * 4 * NPARTS, 0);
    // Scan row structure (V2; row boundaries are the same in the CSR and the
    // kpos-sorted layout): per wave and slot the lanes whose slot starts / ends
    // a row, and (min-sum) parks its tail aggregate (lane masks the scan tests
    // as scalar registers),
    // and per lane the slot mask of each row it starts (bit 63: the row
    // continues into the next lane) for the row parities of the decisions.
    std::vector<uint64_t> row_sem, row_rmask;
    int nst_max = 0;
    auto build_meta = [&](bool sorted, std::vector<uint32_t> &mt, std::vector<uint64_t> &vnm,
                          std::vector<uint32_t> &mt2, std::vector<uint64_t> &vex) -> int {
        const bool rowstruct = v2 && !sorted && g->split_k <= 1 && g->v2RG == 0 && S4 <= 63;
        std::vector<std::vector<uint64_t>> rm(rowstruct ? T : 0);
        if (rowstruct) row_sem.assign((size_t)W * S4 * 4, 0);
        mt.assign((size_t)G4 * TS * 4 * NPARTS, 0);
        mt2.assign(g->n_hd ? (size_t)G4 * TS * 4 * NPARTS : 0, 0);
        vnm.assign(v2 ? (size_t)W * g->dv_max : 0, 0);
        vex.assign(v2 ? (size_t)W * g->dv_max * S4 : 0, 0);
        perm = ledge;
        if (sorted)
            for (int j = 0; j < m; ++j)
                std::stable_sort(perm.begin() + lrp[j], perm.begin() + lrp[j + 1],
                                 [&](int x, int y) { return kpos[x] < kpos[y]; });
        for (int w = 0; w < W; ++w) {
            const long long wb = v2 ? lrp[g->wave_rows[w]] : 0;
            const long long we = v2 ? lrp[g->wave_rows[w + 1]] : E;
            const int lanes = v2 ? 64 : T;
            const int epl_w = v2 ? std::max<int>((int)((we - wb + 63) / 64), g->max_dc) : EPL;
            for (int li = 0; li < lanes; ++li) {
                const int l = w * 64 + li;
                const long long e0 = wb + (long long)li * epl_w;
                if (v2) lepl[l] = epl_w;
                int head = 0;
                lnst[l] = 0;
                if (e0 < we) {
                    const int r0 = lrow[e0];
                    lrow0[l] = r0;
                    if (e0 != lrp[r0]) head = lhead[l] = lrp[r0 + 1] - (int)e0;
                }
                int prev_row = -1;
                for (int k = 0; k < (v2 ? G4 * 4 : epl_w); ++k) {
                    const long long e = e0 + k;  // position in the row-major edge list
                    uint32_t wd;
                    if (k >= epl_w || e >= we) {
                        if (!v2) break;
                        wd = DUMMY;
                        if (sorted && vng_h) vng_meta2[midx(l, k)] = (uint32_t)((vng_chunks + li) * 4);
                        // register-shape bit gather: dummy slots record into the
                        // spare word past the per-bit bytes (V2Layout::syn)
                        if (sorted && !vng_rec.empty()) vng_rec[midx(l, k)] = (uint32_t)((n + 3) & ~3);
                    } else {
                        const int j = lrow[e];
                        const int ed = perm[e];  // the edge at that position
                        wd = (uint32_t)colL[ed] | ((uint32_t)kpos[ed] << META_KPOS_SHIFT) | META_VALID;
                        if (v2) {
                            vnm[(size_t)w * g->dv_max + kpos[ed]] |= 1ull << k;
                            vex[((size_t)w * g->dv_max + kpos[ed]) * S4 + k] |= 1ull << li;
                        }
                        if (sorted && vng_h) vng_meta2[midx(l, k)] = (uint32_t)(P0[col_idx[ed]] + kpos[ed]);
                        if (sorted && !vng_rec.empty() && kpos[ed] < 4) {
                            const uint32_t c = (uint32_t)colL[ed];
                            vng_rec[midx(l, k)] = (c & ~3u) | ((((c & 3u) << 3) + 2u * (uint32_t)kpos[ed]) << 16);
                        }
                        if (g->n_hd && kpos[ed] >= g->vn_k0)
                            mt2[midx(l, k)] =
                                (uint32_t)(stage_off[kpos[ed]] + rank[col_idx[ed]]);
                        if (e == lrp[j]) {
                            wd |= META_START;
                            ++lnst[l];
                            if (rowstruct) {
                                row_sem[((size_t)w * S4 + k) * 4] |= 1ull << li;
                                // slots of this row in the lane; bit 63 when it runs past the lane
                                const long long last = std::min<long long>(lrp[j + 1] - 1, e0 + epl_w - 1);
                                uint64_t msk = 0;
                                for (long long q = e; q <= last; ++q) msk |= 1ull << (q - e0);
                                if (lrp[j + 1] - 1 > e0 + epl_w - 1) msk |= 1ull << 63;
                                rm[l].push_back(msk);
                            }
                        }
                        if (e == lrp[j + 1] - 1 && !(v2 && k < head)) {
                            wd |= META_END;
                            if (rowstruct) row_sem[((size_t)w * S4 + k) * 4 + 1] |= 1ull << li;
                        }
                        if (k > 0 && j != prev_row && j != prev_row + 1)
                            return fail(QLDPC_EUNSUP, "empty check rows between non-empty rows are not supported");
                        prev_row = j;
                    }
                    mt[midx(l, k)] = wd;
                    // min-sum: a lane's tail aggregate (a row begun in the lane
                    // before) is parked at slot `head` — its first START, or a
                    // dummy slot when the wave's edges end with the tail
                    if (rowstruct && head > 0 && k == head && k < S4)
                        row_sem[((size_t)w * S4 + k) * 4 + 2] |= 1ull << li;
                }
            }
        }
        if (rowstruct) {
            for (auto &v : rm) nst_max = std::max(nst_max, (int)v.size());
            row_rmask.assign((size_t)std::max(nst_max, 1) * T, 0);
            for (int l = 0; l < T; ++l)
                for (size_t j = 0; j < rm[l].size(); ++j) row_rmask[j * T + l] = rm[l][j];
        }
        return QLDPC_OK;
    };
    // Occurrence pairing (unsorted adjacency, v1 global-slot layout: edge e at
    // lane e / EPL, slot e % EPL, message index slot * T + lane).  The VN loop
    // (:109-120) visits bit i's checks in bit_nodes order; its jj-th visit of
    // check r fills r's next input slot with total[i] - c2b[i][jj], and
    // c2b[i][jj] is the message of the jj-th check (in check order) holding i
    // (:67-69).  pair_src / pair_col: per input slot, that message's index and i.
    std::vector<int32_t> pair_src, pair_col;
    if (g->paired) {
        if (v2) return fail(QLDPC_EUNSUP, "occurrence pairing needs the v1 layout");
        auto aidx = [&](int e) { return (e % EPL) * T + e / EPL; };
        std::vector<int> cbase(n + 1, 0);
        for (int i = 0; i < n; ++i) cbase[i + 1] = cbase[i] + dv[i];
        std::vector<int> edge_of(E);  // (bit, occurrence rank) -> edge
        for (int e = 0; e < E; ++e) edge_of[cbase[col_idx[e]] + kpos[e]] = e;
        std::vector<int32_t> cp(cbase.begin(), cbase.end()), ri(E);
        if (col_ptr && row_idx) {
            cp.assign(col_ptr, col_ptr + n + 1);
            ri.assign(row_idx, row_idx + E);
        } else {  // bit_nodes = the ascending transpose
            std::vector<int> fill(n, 0);
            for (int j = 0; j < m; ++j)
                for (int e = row_ptr[j]; e < row_ptr[j + 1]; ++e) ri[cbase[col_idx[e]] + fill[col_idx[e]]++] = j;
        }
        pair_src.assign((size_t)EPL * T, 0);
        pair_col.assign((size_t)EPL * T, 0);
        std::vector<int> bpos(m, 0);
        for (int i = 0; i < n; ++i)
            for (int jj = 0; jj < dv[i]; ++jj) {
                const int r = ri[cp[i] + jj];
                const int e_dst = row_ptr[r] + bpos[r]++;
                pair_src[aidx(e_dst)] = aidx(edge_of[cbase[i] + jj]);
                pair_col[aidx(e_dst)] = i;
            }
    }
    std::vector<int32_t> row_orig(v2 ? g->row_order : std::vector<int>());
    g->vng = !vn_rows.empty();
    std::vector<uint32_t> meta_ms, meta2, meta2_ms;
    std::vector<uint64_t> vnm, vnm_ms, vex, vex_ms;
    int brc = build_meta(false, meta, vnm, meta2, vex);
    if (!brc && v2) brc = build_meta(true, meta_ms, vnm_ms, meta2_ms, vex_ms);
    if (brc) return brc;
    // Split frames' exchange layout (DecodeArgs::xoff): each staged term's
    // region is (owner part of its bit, chunk, kpos); inside a region the terms
    // follow (writer wave, slot, lane), so the stage position of every slot is
    // assigned walking the slots in that order.  Region sizes depend only on
    // the edges, so both slot layouts (CSR, kpos-sorted) share xoff.
    std::vector<int32_t> xoff;
    std::vector<uint16_t> xbit, xbit_ms;
    if (v2 && g->split_k > 1 && g->split_cb > 0) {
        const int K = g->split_k, NC = g->split_nc, CB = g->split_cb, D = g->dv_max;
        std::vector<int32_t> reg0(n), lbit(n);
        for (int p = 0; p < K; ++p) {
            const int lo = (int)((long long)n * p / K), hi = (int)((long long)n * (p + 1) / K);
            for (int b = lo; b < hi; ++b) {
                const int c = (b - lo) / CB;
                reg0[b] = (p * NC + c) * D;
                lbit[b] = (b - lo) - c * CB;
            }
        }
        const size_t NR = (size_t)K * NC * D;
        std::vector<long long> fill(NR + 1, 0);
        for (int e = 0; e < E; ++e) ++fill[(size_t)reg0[col_idx[e]] + kpos[e] + 1];
        for (size_t r = 0; r < NR; ++r) fill[r + 1] += fill[r];
        if (fill[NR] != g->stage_doubles) return fail(QLDPC_EUNSUP, "split exchange layout: term count");
        xoff.assign(fill.begin(), fill.end());
        fill.pop_back();
        // Order inside a region: (writer part, slot group of four, wave, slot,
        // lane) — the 16 waves of a part, which run the message pass roughly
        // in step, fill one run per region and slot group together, so a
        // region has one or two open L2 lines per part instead of one per
        // wave.  QLDPC_SPLIT_XORDER=0: (wave, slot, lane), one run per wave (A/B).
        const bool grouped = env_int("QLDPC_SPLIT_XORDER", 1) != 0;
        const int WPp = REG_TSTRIDE / 64;  // waves per part
        auto assign = [&](const std::vector<uint32_t> &mt, std::vector<uint32_t> &mt2, std::vector<uint16_t> &xb) {
            std::vector<long long> pos(fill);
            xb.assign((size_t)g->stage_doubles, 0);
            auto place = [&](int w, int k) {
                for (int li = 0; li < 64; ++li) {
                    const size_t i = midx(w * 64 + li, k);
                    const uint32_t kp = (mt[i] >> META_KPOS_SHIFT) & META_KPOS_MASK;
                    if (kp == META_KPOS_MASK) continue;  // dummy slot
                    const int b = (int)(mt[i] & META_COL_MASK);
                    const long long q = pos[(size_t)reg0[b] + kp]++;
                    mt2[i] = (uint32_t)q;
                    xb[(size_t)q] = (uint16_t)lbit[b];
                }
            };
            if (grouped) {
                for (int p = 0; p < K; ++p)
                    for (int k0 = 0; k0 < S4; k0 += 4)
                        for (int w = p * WPp; w < std::min(W, (p + 1) * WPp); ++w)
                            for (int k = k0; k < k0 + 4; ++k) place(w, k);
            } else {
                for (int w = 0; w < W; ++w)
                    for (int k = 0; k < S4; ++k) place(w, k);
            }
        };
        assign(meta, meta2, xbit);
        assign(meta_ms, meta2_ms, xbit_ms);
    }
    g->nst_max = row_sem.empty() ? 0 : nst_max;
    if (v2 && qldpc_diag_env("QLDPC_DEBUG_PLAN")) {  // host-side plan statistics on stderr
        auto visited = [&](const std::vector<uint64_t> &v) {
            long long s = 0;
            for (int w = 0; w < W; ++w)
                for (int kk = 1; kk < g->dv_max; ++kk) s += __builtin_popcountll(v[(size_t)w * g->dv_max + kk]);
            return s;
        };
        long long full = 0;
        for (int w = 0; w < W; ++w) full += (long long)(g->dv_max - 1) * lepl[w * 64];
        fprintf(stderr, "{\"plan\": {\"waves\": %d, \"slots_reg\": %d, \"slots_scratch\": %d, \"epl_max\": %d, "
                        "\"dv_max\": %d, \"vn_slot_visits_csr\": %lld, \"vn_slot_visits_kpos_sorted\": %lld, "
                        "\"vn_slot_visits_unmasked\": %lld, \"rows_global_ms\": %d, \"rows_lds_ms\": %d, "
                        "\"rows_lds_waves_ms\": %d, \"split_k\": %d, \"split_cb\": %d, \"split_nc\": %d}}\n",
                W, g->v2R, g->v2RG, g->EPL, g->dv_max, visited(vnm), visited(vnm_ms), full, (int)g->rows_global_ms,
                g->rows_lds_ms, g->rows_lds_waves_ms, g->split_k, g->split_cb, g->split_nc);
        fprintf(stderr, "{\"relabel\": {\"excess_before\": %lld, \"excess_after\": %lld, \"cycles_before\": %lld, "
                        "\"cycles_after\": %lld}}\n",
                g->relabel_stats[0], g->relabel_stats[1], g->relabel_stats[2], g->relabel_stats[3]);
    }
    // Row-ELL (slot-major) for syndrome evaluation.
    const int dcm = std::max(1, g->max_dc);
    std::vector<int32_t> ell((size_t)dcm * std::max(m, 1), 0), rdeg(std::max(m, 1), 0);
    for (int j = 0; j < m; ++j) {
        rdeg[j] = row_ptr[j + 1] - row_ptr[j];
        for (int k = 0; k < rdeg[j]; ++k) ell[(size_t)k * m + j] = col_idx[row_ptr[j] + k];
    }

    std::vector<int32_t> ell_lab, col_orig;
    if (!g->col_lab.empty()) {
        ell_lab = ell;
        for (int j = 0; j < m; ++j)
            for (int k = 0; k < rdeg[j]; ++k) ell_lab[(size_t)k * m + j] = g->col_lab[ell[(size_t)k * m + j]];
        col_orig.resize(n);
        for (int i = 0; i < n; ++i) col_orig[g->col_lab[i]] = i;
    }
    if (host_only) {
        *out = g.release();
        return QLDPC_OK;
    }

    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    std::vector<int> devices;
    if (device_list) {
        for (int d : *device_list)
            if (d < 0 || d >= ndev) return fail(QLDPC_EINVAL, "device list names a device that does not exist");
        devices = *device_list;
    } else if (device_mask == 0) {
        int cur = 0;
        HIP_TRY(hipGetDevice(&cur));
        devices.push_back(cur);
    } else {
        for (int d = 0; d < 31; ++d)
            if (device_mask & (1 << d)) {
                if (d >= ndev) return fail(QLDPC_EINVAL, "device_mask names a device that does not exist");
                devices.push_back(d);
            }
    }
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    for (int d : devices) {
        auto dg = std::make_unique<DeviceGraph>();
        dg->device = d;
        HIP_TRY(hipSetDevice(d));
        HIP_TRY(hipDeviceGetAttribute(&dg->num_cus, hipDeviceAttributeMultiprocessorCount, d));
        int rc;
        if ((rc = upload(&dg->slot_meta, meta)) || (rc = upload(&dg->slot_meta_ms, meta_ms)) ||
            (rc = upload(&dg->vn_mask, vnm)) || (rc = upload(&dg->vn_mask_ms, vnm_ms)) ||
            (rc = upload(&dg->vn_exec, vex)) || (rc = upload(&dg->vn_exec_ms, vex_ms)) ||
            (rc = upload(&dg->slot_meta2, meta2)) || (rc = upload(&dg->slot_meta2_ms, meta2_ms)) ||
            (rc = upload(&dg->hd_bits, hd_bits)) || (rc = upload(&dg->hd_dv, hd_dv)) ||
            (rc = upload(&dg->stage_off, stage_off)) || (rc = upload(&dg->row_orig, row_orig)) ||
            (rc = upload(&dg->part_row0, g->part_row0)) || (rc = upload(&dg->xoff, xoff)) ||
            (rc = upload(&dg->xbit, xbit)) || (rc = upload(&dg->xbit_ms, xbit_ms)) ||
            (rc = upload(&dg->lane_row0, lrow0)) || (rc = upload(&dg->wave_rows, g->wave_rows)) ||
            (rc = upload(&dg->lane_head, lhead)) || (rc = upload(&dg->lane_nst, lnst)) ||
            (rc = upload(&dg->lane_epl, lepl)) || (rc = upload(&dg->ell_col, ell)) ||
            (rc = upload(&dg->row_deg, rdeg)) || (rc = upload(&dg->iso_bits, iso)) ||
            (rc = upload(&dg->vn_rows, vn_rows)) || (rc = upload(&dg->vng_bits, vng_bits)) ||
            (rc = upload(&dg->vng_meta2, vng_meta2)) || (rc = upload(&dg->row_sem, row_sem)) ||
            (rc = upload(&dg->vng_rec, vng_rec)) ||
            (rc = upload(&dg->row_rmask, row_rmask)) ||
            (g->paired && ((rc = upload(&dg->pair_src, pair_src)) || (rc = upload(&dg->pair_col, pair_col)))) ||
            (!col_orig.empty() && ((rc = upload(&dg->col_orig, col_orig)) || (rc = upload(&dg->col_lab, g->col_lab)) ||
                                   (rc = upload(&dg->ell_lab, ell_lab))))) {
            (void)hipSetDevice(prev);
            return rc;
        }
        g->devs.push_back(std::move(dg));
    }
    HIP_TRY(hipSetDevice(prev));
    *out = g.release();
    return QLDPC_OK;
}

DeviceGraph *find_dev(qldpc_graph *g, int device) {
    for (auto &d : g->devs)
        if (d->device == device) return d.get();
    return nullptr;
}

int check_params(const qldpc_params *p) {
    if (!p) return fail(QLDPC_EINVAL, "params is NULL");
    if (p->algorithm < 0 || p->algorithm > 5) return fail(QLDPC_EINVAL, "algorithm must be 0..5");
    if (p->max_iterations < 1) return fail(QLDPC_EINVAL, "max_iterations must be >= 1");
    if (p->thr_enabled && !(p->thr > 0.)) return fail(QLDPC_EINVAL, "threshold must be > 0 when enabled");
    return QLDPC_OK;
}

// Per-workgroup scratch of the V2 kernels: overflow message slots, then the VN stage.
// Hybrid min-sum with rows in global scratch: their offset (16-byte aligned).
long long v2_rows_offset(const qldpc_graph &g) {
    return ((long long)g.v2RG * REG_TSTRIDE + g.stage_doubles + 1) / 2 * 2;
}

// v1: the kernel's scratch, plus (occurrence pairing) a slot-major b2c buffer
long long v1_scratch_doubles(const qldpc_graph &g) {
    return scratch_doubles_for(g.variant, g.n, g.m, g.T, g.EPL) + (g.paired ? (long long)g.EPL * g.T : 0);
}

// Relabelled graphs: a non-paletted frame's llr[] in label order, per workgroup
// (DecodeArgs::llr_lab_wg_offset), after everything else; -1: not relabelled.
long long v2_llr_lab_offset(const qldpc_graph &g) {
    if (g.split_k > 1 || g.col_lab.empty()) return -1;
    const long long end = g.rows_global_ms ? v2_rows_offset(g) + 2LL * g.m
                                           : (long long)g.v2RG * REG_TSTRIDE + g.stage_doubles;
    return (end + 31) / 32 * 32;
}

long long v2_scratch_doubles(const qldpc_graph &g) {
    // split frames: the stage is per frame (Workspace::gstage); only the
    // scratch message slots of a V2_RG_SPLIT plan are per workgroup
    if (g.split_k > 1) return g.v2RG > 0 ? (long long)g.v2RG * REG_TSTRIDE : 32;
    long long end = g.rows_global_ms ? v2_rows_offset(g) + 2LL * g.m
                                     : (long long)g.v2RG * REG_TSTRIDE + g.stage_doubles;
    if (v2_llr_lab_offset(g) >= 0) end = v2_llr_lab_offset(g) + g.n;
    return (end + 31) / 32 * 32;
}

// Per-stream workspace of a device graph, created on first use.
Workspace *workspace(DeviceGraph *dg, hipStream_t stream) { return &dg->ws[(void *)stream]; }

// Ensure the workspace holds V2 frame codes for `batch` frames (caller holds dg->mu).
int ensure_codes(qldpc_graph *g, Workspace *w, int batch, hipStream_t stream) {
    if ((size_t)batch <= w->code_frames) return QLDPC_OK;
    HIP_TRY(hipStreamSynchronize(stream));
    (void)hipFree(w->codes);
    (void)hipFree(w->palette);
    (void)hipFree(w->pal_ok);
    w->codes = nullptr; w->palette = nullptr; w->pal_ok = nullptr; w->code_frames = 0;
    const size_t nc = (size_t)(g->n + 3) / 4;
    HIP_TRY(hipMalloc(&w->codes, (size_t)batch * nc));
    HIP_TRY(hipMalloc(&w->palette, (size_t)batch * 4 * sizeof(double)));
    HIP_TRY(hipMalloc(&w->pal_ok, (size_t)batch));
    w->code_frames = (size_t)batch;
    return QLDPC_OK;
}

// The device frame builders stage the frame's keys in LDS as bit words
// (decoder.hpp build_frames_lds / build_frames_ra_lds): refuse larger graphs
// with a message instead of a launch error.  (Plain frames: n <= 655,360;
// rate-adapted: n <= ~436k; the reference's codes stop at n = 102,400.)
int frame_builder_fits(const qldpc_graph *g, int n_punct /* < 0: plain frames */) {
    const size_t lds = n_punct < 0 ? build_frames_lds(g->n) : build_frames_ra_lds(g->n, n_punct);
    if (lds <= LDS_MAX_BYTES) return QLDPC_OK;
    return fail(QLDPC_EUNSUP, "n = " + std::to_string(g->n) + ": the device frame builder keeps the frame's keys in " +
                                  "LDS (" + std::to_string(lds) + " bytes > " + std::to_string(LDS_MAX_BYTES) +
                                  "); decode such frames through qldpc_decode_batch[_device] with host-built LLRs");
}

// Split frames in flight per physical device.  A part group forms from K
// workgroups of ONE launch resident on one XCD (the claim counter is per launch
// and XCD).  Two persistent split launches that are each only partly resident
// could wait on each other's workgroups until the group timeout — but only if
// each holds fewer than K of an XCD's S workgroup slots, which cannot happen
// when two launches fill the XCD and 2 (K - 1) < S: one of them then has >= K
// there, its groups complete, and its workgroups leave when its frames run out.
// So a split launch (hipStreamWaitEvent, on the GPU) always waits for the split
// launch two before it on its device (at most two in flight), and also for
// the previous one unless both have the same shape (K, part size, LDS: the
// same S) with 2 (K - 1) < S and batches of at most 2048 frames
// (every shipped plan: K <= 16 of S = 64 8-wave or 32 16-wave slots).  The
// 2-stream bench and the batch seam then still start batch i + 1's frames in
// batch i's tail.  One-workgroup frames have no such coupling.
struct SplitSerial {
    std::mutex mu;
    hipEvent_t ev[2] = {nullptr, nullptr};  // the last two split launches' ends
    long long shape[2] = {-1, -1};          // K, part lanes and LDS bytes of that launch
    bool overlap_ok[2] = {false, false};    // 2 (K - 1) < S for that launch
    int last = -1;                          // ev[last] is the most recent (-1: none yet)
};
SplitSerial &split_serial(int device) {
    static std::mutex mu;
    static std::map<int, std::unique_ptr<SplitSerial>> per_device;
    std::lock_guard<std::mutex> lk(mu);
    auto &p = per_device[device];
    if (!p) p.reset(new SplitSerial);
    return *p;
}

// Split frames: after the stream is idle, fail loudly if a part group timed
// out waiting for its members (the kernel never hangs on it; results are void).
int split_check(qldpc_graph *g, DeviceGraph *dg, hipStream_t stream) {
    if (g->variant != VAR_V2 || g->split_k <= 1) return QLDPC_OK;
    int *ctl = nullptr;
    {
        std::lock_guard<std::mutex> lk(dg->mu);  // ws is shared with other streams' calls
        ctl = workspace(dg, stream)->split_ctl;
    }
    if (!ctl) return QLDPC_OK;
    int err = 0;
    HIP_TRY(hipMemcpy(&err, ctl + 16, sizeof(int), hipMemcpyDeviceToHost));
    if (err) return fail(QLDPC_EHIP, "split frame: a part group failed to meet (results void)");
    return QLDPC_OK;
}

// Enqueue the decoder for `batch` device-resident frames on `stream`.  For the
// V2 kernel the frames' palette + codes are taken from the stream's workspace
// when `codes_ready` (written by build_frames), else computed here from llr.
// The decode kernel waits for `before_decode` when given (the kernels that
// prepare it do not).
int decode_on(qldpc_graph *g, DeviceGraph *dg, const qldpc_params *p, int batch, const double *llr,
              const uint8_t *synd, uint8_t *bits, uint32_t *iters, uint8_t *ok, double *post,
              hipStream_t stream, bool codes_ready = false, uint64_t *frame_clk = nullptr,
              hipEvent_t before_decode = nullptr) {
    if (batch == 0) return QLDPC_OK;
    const int alg = p->algorithm;
    const bool v2 = g->variant == VAR_V2;
    const size_t lds = lds_of(*g, alg);
    Workspace *w;
    int wgs;
    {
        std::lock_guard<std::mutex> lk(dg->mu);
        if (dg->occ[alg] == 0) {
            int b = 0;
            if (v2) HIP_TRY(occupancy_v2(g->v2R, g->v2RG, g->split_k, alg, block_threads(*g), lds, &b));
            else HIP_TRY(occupancy(g->variant, alg, g->T, lds, &b));
            if (b <= 0) return fail(QLDPC_EUNSUP, "decoder kernel cannot be resident with this graph shape");
            dg->occ[alg] = b;
        }
        wgs = std::min(batch, dg->occ[alg] * dg->num_cus);
        // split frames: every workgroup of the device (each XCD must hold whole
        // part groups; the claim protocol needs >= split_k of them per XCD)
        if (v2 && g->split_k > 1) {
            wgs = dg->occ[alg] * dg->num_cus;
            // QLDPC_SPLIT_WGS (A/B): fewer workgroups, so fewer frames share an
            // XCD's L2 (whole XCD rounds of 8; every XCD keeps >= split_k)
            const int lim = env_int("QLDPC_SPLIT_WGS", 0);
            if (lim >= 8 * g->split_k && lim < wgs) wgs = lim - lim % 8;
        }
        w = workspace(dg, stream);
        if (!w->counter) HIP_TRY(hipMalloc(&w->counter, 64));
        if (v2) {
            if (codes_ready && (size_t)batch > w->code_frames)
                return fail(QLDPC_EINVAL, "frame codes were not built for this batch");
            int rc = ensure_codes(g, w, batch, stream);
            if (rc) return rc;
            if (g->split_k > 1 && (size_t)batch > w->split_frames) {
                HIP_TRY(hipStreamSynchronize(stream));
                (void)hipFree(w->split_ctl);
                (void)hipFree(w->gtotal);
                (void)hipFree(w->gstage);
                w->split_ctl = nullptr; w->gtotal = nullptr; w->gstage = nullptr; w->split_frames = 0;
                const size_t slots = (size_t)batch + 64;
                HIP_TRY(hipMalloc(&w->split_ctl, (32 + 3 * 16 * slots) * sizeof(int)));
                HIP_TRY(hipMalloc(&w->gtotal, (size_t)batch * (g->n + 1) * sizeof(double)));
                HIP_TRY(hipMalloc(&w->gstage, (size_t)batch * std::max<long long>(1, g->stage_doubles) * sizeof(double)));
                w->split_frames = (size_t)batch;
            }
        }
        if ((size_t)batch > w->order_frames) {
            HIP_TRY(hipStreamSynchronize(stream));
            (void)hipFree(w->fweight);
            (void)hipFree(w->forder);
            w->fweight = nullptr; w->forder = nullptr; w->order_frames = 0;
            HIP_TRY(hipMalloc(&w->fweight, (size_t)batch * sizeof(int32_t)));
            HIP_TRY(hipMalloc(&w->forder, (size_t)batch * sizeof(int32_t)));
            w->order_frames = (size_t)batch;
        }
        {
            const long long per = v2 ? v2_scratch_doubles(*g) : v1_scratch_doubles(*g);
            const size_t need = (size_t)per * (size_t)wgs;
            if (need > w->scratch_doubles) {
                if (w->scratch) {
                    HIP_TRY(hipStreamSynchronize(stream));
                    HIP_TRY(hipFree(w->scratch));
                    w->scratch = nullptr;
                }
                HIP_TRY(hipMalloc(&w->scratch, need * sizeof(double)));
                w->scratch_doubles = need;
            }
        }
    }
    DecodeArgs a{};
    a.n = g->n; a.m = g->m; a.E = g->E; a.T = block_threads(*g); a.EPL = g->EPL; a.dv_max = g->dv_max; a.max_dc = g->max_dc;
    a.slot_meta = dg->slot_meta; a.lane_row0 = dg->lane_row0; a.lane_head = dg->lane_head;
    a.lane_nst = dg->lane_nst; a.lane_epl = dg->lane_epl;
    if (v2 && alg >= 2) a.slot_meta = dg->slot_meta_ms;
    a.vn_mask = (v2 && alg >= 2) ? dg->vn_mask_ms : dg->vn_mask;
    a.vn_exec = (v2 && alg >= 2) ? dg->vn_exec_ms : dg->vn_exec;
    a.ell_col = dg->ell_col; a.row_deg = dg->row_deg;
    a.alg = alg; a.max_it = p->max_iterations; a.thr_on = p->thr_enabled ? 1 : 0;
    a.thr = p->thr; a.primary = p->primary; a.secondary = p->secondary;
    {
        const bool norm = alg == 2 || alg == 4, adapt = alg == 4 || alg == 5;
        const auto fine = [&](double f) { return norm ? (std::fabs(f) <= 1.0) : (f >= 0.0); };  // NaN: not fine
        a.ms_clip_later = (fine(p->primary) && (!adapt || fine(p->secondary))) ? 0 : 1;
    }
    {
        const double lim = (a.thr_on && p->thr < 44.0) ? p->thr : 44.0;
        a.spa_tlim = std::tanh(lim / 2.);
        a.spa_ctop = 2. * std::atanh(0x1.fffffffffffffp-1);
    }
    a.batch = batch; a.llr = llr; a.synd = synd; a.bits = bits; a.iters = iters; a.ok = ok; a.post = post;
    a.frame_counter = w->counter;
    a.scratch = w->scratch;
    a.scratch_wg_doubles = v2 ? v2_scratch_doubles(*g) : v1_scratch_doubles(*g);
    if (!v2 && g->paired) {
        a.pair_src = dg->pair_src;
        a.pair_col = dg->pair_col;
        a.pair_buf_off = scratch_doubles_for(g->variant, g->n, g->m, g->T, g->EPL);
    }
    a.hd_uniform_dv = g->hd_uniform_dv;
    a.vn_k0 = g->vn_k0; a.n_hd = g->n_hd; a.hd_bits = dg->hd_bits; a.hd_dv = dg->hd_dv; a.stage_off = dg->stage_off;
    a.slot_meta2 = (v2 && alg >= 2) ? dg->slot_meta2_ms : dg->slot_meta2;
    a.stage_wg_offset = (long long)g->v2RG * REG_TSTRIDE;
    a.rows_wg_offset = (v2 && g->rows_global_ms && alg >= 2) ? v2_rows_offset(*g) : -1;
    a.rows_lds = (v2 && g->rows_global_ms && alg >= 2) ? g->rows_lds_ms : g->m;
    a.rows_lds_waves = (v2 && g->rows_global_ms && alg >= 2) ? g->rows_lds_waves_ms : (g->T / 64);
    a.wave_rows = dg->wave_rows;
    // the rows kept in global scratch fit the totals region below total[n]
    // (dead between the scan and the bit gather): their waves' message pass
    // reads them from an LDS copy (QLDPC_ROWS_COPY=0: from L2, A/B)
    a.rows_copy = (a.rows_wg_offset >= 0 && (long long)(g->m - a.rows_lds) * 16 <= (long long)g->n * 8 &&
                   env_int("QLDPC_ROWS_COPY", 1))
                      ? 1 : 0;
    a.row_orig = dg->row_orig;
    a.col_orig = dg->col_orig;
    a.col_lab = dg->col_lab;
    a.llr_lab_wg_offset = (v2 && dg->col_orig) ? v2_llr_lab_offset(*g) : -1;
    a.frame_clk = frame_clk;
    a.row_sem = (v2 && g->nst_max > 0) ? dg->row_sem : nullptr;
    a.row_rmask = (v2 && g->nst_max > 0) ? dg->row_rmask : nullptr;
    a.nst_max = g->nst_max;
    a.split_k = v2 ? g->split_k : 1;
    if (v2 && g->split_k > 1) {
        const int slots = (int)w->split_frames + 64;
        a.split_mrows = g->split_mrows;
        a.split_slots = slots;
        a.part_row0 = dg->part_row0;
        a.split_claim = w->split_ctl;
        a.split_err = w->split_ctl + 16;
        a.split_pub = w->split_ctl + 32;
        a.split_sync = a.split_pub + 16 * slots;
        a.split_mis = a.split_sync + 16 * slots;
        a.gtotal = w->gtotal;
        a.gstage = w->gstage;
        a.stage_frame_doubles = g->stage_doubles;
        a.split_cb = g->split_cb;
        a.split_nc = g->split_nc;
        a.xoff = g->split_cb > 0 ? dg->xoff : nullptr;
        a.xbit = alg >= 2 ? dg->xbit_ms : dg->xbit;
        HIP_TRY(hipMemsetAsync(w->split_ctl, 0, (32 + 3 * 16 * (size_t)slots) * sizeof(int), stream));
    }
    a.nc = (g->n + 3) / 4;
    a.codes = w->codes; a.palette = w->palette; a.pal_ok = w->pal_ok;
    a.n_iso = g->n_iso; a.iso_bits = dg->iso_bits; a.v2R = g->v2R; a.v2RG = g->v2RG;
    {  // min-sum bit gather where the shape allows it (QLDPC_VNG=0: VN phases instead)
        const char *e = qldpc_diag_env("QLDPC_VNG");
        const bool off = e && std::strcmp(e, "0") == 0;
        if (v2 && g->vng && !off && v2_vng_ok(alg, g->v2R, g->v2RG, a.split_k, g->dv_max, g->m)) {
            a.vn_rows = reinterpret_cast<const uint2 *>(dg->vn_rows);
            if (g->v2RG > 0) {
                a.vng_bits = reinterpret_cast<const uint2 *>(dg->vng_bits);
                a.slot_meta2 = dg->vng_meta2;
            } else {
                a.slot_meta2 = dg->vng_rec;
            }
        }
        if (a.rows_wg_offset >= 0 && !a.vn_rows)
            return fail(QLDPC_EUNSUP, "this code's min-sum row aggregates need the bit gather (QLDPC_VNG=0 given)");
    }
    if (v2 && !codes_ready)  // (relabelled graphs: the kernel reads a non-paletted frame by label)
        HIP_TRY(launch_palettize(g->n, a.nc, batch, llr, w->codes, w->palette, w->pal_ok, dg->col_orig, stream));
    {  // claim order: hardest-looking frames first (order.hip; QLDPC_ORDER=0: index order).
        // It only schedules — results never depend on it — so a shape it cannot
        // run (LDS beyond the device limit) decodes in index order instead.
        const char *e = qldpc_diag_env("QLDPC_ORDER");
        if (!(e && std::strcmp(e, "0") == 0) && batch > 1) {
            // (relabelled graphs: the frame codes are in label order, so is the row-ELL it reads)
            const hipError_t oe = launch_frame_order(g->n, g->m, dg->col_orig ? dg->ell_lab : dg->ell_col,
                                                     dg->row_deg, batch, synd, llr, v2 ? w->codes : nullptr,
                                                     w->palette, w->pal_ok, w->fweight, w->forder, dg->col_orig,
                                                     stream);
            if (oe == hipSuccess) a.frame_order = w->forder;
            else (void)hipGetLastError();  // clear the sticky launch error; index order
        }
        w->order_count = a.frame_order ? batch : 0;
    }
    HIP_TRY(hipMemsetAsync(w->counter, 0, sizeof(int), stream));
#ifdef QL_PHASE_STAMPS
    const size_t nst = (size_t)wgs * (block_threads(*g) / 64) * NUM_STAMPS;
    uint64_t *d_st = nullptr;
    HIP_TRY(hipMalloc(&d_st, nst * sizeof(uint64_t)));
    HIP_TRY(hipMemsetAsync(d_st, 0, nst * sizeof(uint64_t), stream));
    a.stamps = d_st;
#endif
    std::unique_lock<std::mutex> split_lk;
    SplitSerial *ser = nullptr;
    int ser_slot = 0;
    bool ser_ok = false;
    long long ser_shape = -1;
    if (v2 && g->split_k > 1) {  // split launches in flight per device (above)
        ser = &split_serial(dg->device);
        split_lk = std::unique_lock<std::mutex>(ser->mu);
        for (auto &e : ser->ev)
            if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        const int slots_per_xcd = wgs / 8;  // (8 XCDs; every workgroup of the device is launched)
        // (batches of <= 2048 frames: a group that waits for the other launch to
        // leave its XCD waits at most that launch's run — at 50 iterations of a
        // C4 frame ~0.6 s — well inside the group timeout of ~4 s)
        ser_ok = 2 * (g->split_k - 1) < slots_per_xcd && batch <= 2048;
        ser_shape = ((long long)g->split_k << 48) | ((long long)g->split_pl << 32) | (long long)lds;
        if (ser->last >= 0) {
            const int prev = ser->last, older = prev ^ 1;
            if (ser->shape[older] >= 0) HIP_TRY(hipStreamWaitEvent(stream, ser->ev[older], 0));
            if (!(ser_ok && ser->overlap_ok[prev] && ser->shape[prev] == ser_shape))
                HIP_TRY(hipStreamWaitEvent(stream, ser->ev[prev], 0));
        }
        ser_slot = ser->last < 0 ? 0 : ser->last ^ 1;
    }
    if (g->kernel_timing) {  // (the workspace is per stream: no other call records on these events)
        if (!w->ev0) HIP_TRY(hipEventCreate(&w->ev0));
        if (!w->ev1) HIP_TRY(hipEventCreate(&w->ev1));
        HIP_TRY(hipEventRecord(w->ev0, stream));
    }
    if (before_decode) HIP_TRY(hipStreamWaitEvent(stream, before_decode, 0));
    if (v2) HIP_TRY(launch_decode_v2(a, wgs, lds, stream));
    else HIP_TRY(launch_decode(g->variant, a, wgs, lds, stream));
    if (ser) {
        HIP_TRY(hipEventRecord(ser->ev[ser_slot], stream));
        ser->shape[ser_slot] = ser_shape;
        ser->overlap_ok[ser_slot] = ser_ok;
        ser->last = ser_slot;
        split_lk.unlock();
    }
    if (g->kernel_timing) {
        HIP_TRY(hipEventRecord(w->ev1, stream));
        w->ev_recorded = true;
    }
#ifdef QL_PHASE_STAMPS
    {  // diagnostic: per-phase share of wave time, one JSON line on stderr
        std::vector<uint64_t> h(nst);
        HIP_TRY(hipStreamSynchronize(stream));
        HIP_TRY(hipMemcpy(h.data(), d_st, nst * sizeof(uint64_t), hipMemcpyDeviceToHost));
        (void)hipFree(d_st);
        double tot[NUM_STAMPS] = {0}, all = 0;
        for (size_t i = 0; i < nst; ++i) tot[i % NUM_STAMPS] += (double)h[i];
        for (int i = 0; i < NUM_STAMPS; ++i) all += tot[i];
        std::string js = "{\"phase_stamps\": {";
        for (int i = 0; i < NUM_STAMPS; ++i)
            js += std::string(i ? ", " : "") + "\"" + STAMP_NAMES[i] + "\": " + std::to_string(all > 0 ? tot[i] / all : 0.);
        js += "}, \"wave_cycles_total\": " + std::to_string(all) + "}";
        fprintf(stderr, "%s\n", js.c_str());
    }
#endif
    return QLDPC_OK;
}

// QKD_LDPC's (plan == NULL) or QKD_LDPC_RATE_ADAPT's per-trial window for
// `batch` device-resident trials on `stream` (the current device is dg's):
// frame build, decode, key comparison.  V2 decoders read the frame builder's
// palette codes, so the f64 LLRs are written only into a caller workspace
// (d_llr_ws, nullable); the other decoders read llr[] from it or, when it is
// NULL, from the stream workspace's.
int qkd_ldpc_window(qldpc_graph *g, DeviceGraph *dg, const qldpc_rate_plan *plan, const qldpc_params *p, int batch,
                    const uint8_t *d_alice, const uint8_t *d_bob, const uint8_t *d_punct_alice,
                    const uint8_t *d_punct_bob, const double *d_log_p, uint8_t *d_alice_ext, double *d_llr_ws,
                    uint8_t *d_synd_ws, uint8_t *d_bits_out, uint32_t *d_iters_out, uint8_t *d_synd_ok_out,
                    uint8_t *d_keys_match_out, hipStream_t s, uint64_t *frame_clk = nullptr,
                    hipEvent_t before_decode = nullptr) {
    if (batch == 0) return QLDPC_OK;
    const qldpc_rate_plan::Dev *pd = nullptr;
    if (plan) {
        for (auto &d : plan->devs)
            if (d.device == dg->device) pd = &d;
        if (!pd) return fail(QLDPC_EINVAL, "rate plan does not live on that device");
    }
    const bool v2 = g->variant == VAR_V2;
    uint8_t *codes = nullptr, *pal_ok = nullptr;
    double *palette = nullptr;
    double *llr = d_llr_ws;
    {
        std::lock_guard<std::mutex> lk(dg->mu);
        Workspace *w = workspace(dg, s);
        if (v2) {
            // the frame builder writes the V2 palette + codes straight into the
            // stream's workspace, so the decoder skips the palettize pass
            int r = ensure_codes(g, w, batch, s);
            if (r) return r;
            codes = w->codes; palette = w->palette; pal_ok = w->pal_ok;
        } else if (!llr) {
            if ((size_t)batch > w->llr_ws_frames) {
                HIP_TRY(hipStreamSynchronize(s));
                (void)hipFree(w->llr_ws);
                w->llr_ws = nullptr;
                w->llr_ws_frames = 0;
                HIP_TRY(hipMalloc(&w->llr_ws, (size_t)batch * g->n * sizeof(double)));
                w->llr_ws_frames = (size_t)batch;
            }
            llr = w->llr_ws;
        }
    }
    if (int r = frame_builder_fits(g, plan ? plan->n_punct : -1)) return r;
    if (plan)
        HIP_TRY(launch_build_frames_ra(g->n, g->m, dg->ell_col, dg->row_deg, pd->cls, pd->src, plan->n_punct, batch,
                                       d_alice, d_bob, d_punct_alice, d_punct_bob, d_log_p, d_alice_ext, llr,
                                       d_synd_ws, codes, palette, pal_ok, dg->col_orig, s));
    else
        HIP_TRY(launch_build_frames(g->n, g->m, g->max_dc, dg->ell_col, dg->row_deg, batch, d_alice, d_bob, d_log_p,
                                    llr, d_synd_ws, codes, palette, pal_ok, dg->col_orig, s));
    int r = decode_on(g, dg, p, batch, llr, d_synd_ws, d_bits_out, d_iters_out, d_synd_ok_out, nullptr, s, v2,
                      frame_clk, before_decode);
    if (r) return r;
    // keys_match = arrays_equal(alice[_extended], bob_solution) (:1087, :1216)
    if (d_keys_match_out)
        HIP_TRY(launch_keys_match(batch, g->n, plan ? d_alice_ext : d_alice, d_bits_out, d_keys_match_out, s));
    return QLDPC_OK;
}

template <typename T>
int grow(T **p, size_t count) {
    if (*p) HIP_TRY(hipFree(*p));
    *p = nullptr;
    HIP_TRY(hipMalloc(p, std::max<size_t>(count, 1) * sizeof(T)));
    return QLDPC_OK;
}

}  // namespace

extern "C" {

const char *qldpc_last_error(void) { return g_last_error.c_str(); }

const char *qldpc_version(void) { return "qkd_ldpc_v_amd 0.1.0 (gfx950)"; }

int qldpc_device_count(int32_t *count) {
    if (!count) return fail(QLDPC_EINVAL, "count is NULL");
    int c = 0;
    HIP_TRY(hipGetDeviceCount(&c));
    *count = c;
    return QLDPC_OK;
}

double qldpc_log_p(double qber) { return std::log((1. - qber) / qber); }

int qldpc_load_matrix(const char *path, int32_t format, int32_t *n, int32_t *m, int32_t *nnz, int32_t *row_ptr,
                      int32_t *col_idx, int32_t *col_ptr, int32_t *row_idx, int32_t *is_regular) {
    if (!path || !n || !m || !nnz) return fail(QLDPC_EINVAL, "path/n/m/nnz must not be NULL");
    try {
        const HMatrix H = load_matrix(path, format);
        long long e_rows = 0, e_cols = 0;
        for (const auto &r : H.check_nodes) e_rows += (long long)r.size();
        for (const auto &c : H.bit_nodes) e_cols += (long long)c.size();
        *n = (int32_t)H.bit_nodes.size();
        *m = (int32_t)H.check_nodes.size();
        *nnz = (int32_t)e_rows;
        if (is_regular) *is_regular = H.is_regular ? 1 : 0;
        if (e_rows != e_cols)
            return fail(QLDPC_EINVAL, "check_nodes and bit_nodes hold different edge counts (" +
                                          std::to_string(e_rows) + " vs " + std::to_string(e_cols) + ")");
        if (row_ptr && col_idx) {
            int32_t o = 0;
            for (size_t j = 0; j < H.check_nodes.size(); ++j) {
                row_ptr[j] = o;
                for (int c : H.check_nodes[j]) col_idx[o++] = c;
            }
            row_ptr[H.check_nodes.size()] = o;
        }
        if (col_ptr && row_idx) {
            int32_t o = 0;
            for (size_t i = 0; i < H.bit_nodes.size(); ++i) {
                col_ptr[i] = o;
                for (int r : H.bit_nodes[i]) row_idx[o++] = r;
            }
            col_ptr[H.bit_nodes.size()] = o;
        }
    } catch (const std::exception &e) {
        return fail(QLDPC_EIO, e.what());
    }
    return QLDPC_OK;
}

int qldpc_graph_create(int32_t n, int32_t m, const int32_t *row_ptr, const int32_t *col_idx, int32_t device_mask,
                       qldpc_graph **out) {
    return build_graph(n, m, row_ptr, col_idx, device_mask, out);
}

int qldpc_graph_create_checked(int32_t n, int32_t m, const int32_t *row_ptr, const int32_t *col_idx,
                               const int32_t *col_ptr, const int32_t *row_idx, int32_t device_mask,
                               qldpc_graph **out) {
    if (!row_ptr || !col_idx || !col_ptr || !row_idx) return fail(QLDPC_EINVAL, "NULL adjacency array");
    if (n <= 0 || m < 0) return fail(QLDPC_EINVAL, "invalid graph dimensions");
    // bit_nodes in the caller's order: anything but the ascending transpose of
    // ascending check_nodes rows decodes with the reference's occurrence
    // pairing (build_graph)
    return build_graph(n, m, row_ptr, col_idx, device_mask, out, false, nullptr, col_ptr, row_idx);
}

int qldpc_graph_create_on(int32_t n, int32_t m, const int32_t *row_ptr, const int32_t *col_idx,
                          const int32_t *devices, int32_t ndevices, qldpc_graph **out) {
    if (!devices || ndevices <= 0 || ndevices > 64) return fail(QLDPC_EINVAL, "need 1..64 devices");
    const std::vector<int> list(devices, devices + ndevices);
    return build_graph(n, m, row_ptr, col_idx, 0, out, false, &list);
}

int qldpc_graph_create_checked_on(int32_t n, int32_t m, const int32_t *row_ptr, const int32_t *col_idx,
                                  const int32_t *col_ptr, const int32_t *row_idx, const int32_t *devices,
                                  int32_t ndevices, qldpc_graph **out) {
    if (!row_ptr || !col_idx || !col_ptr || !row_idx) return fail(QLDPC_EINVAL, "NULL adjacency array");
    if (n <= 0 || m < 0) return fail(QLDPC_EINVAL, "invalid graph dimensions");
    if (!devices || ndevices <= 0 || ndevices > 64) return fail(QLDPC_EINVAL, "need 1..64 devices");
    const std::vector<int> list(devices, devices + ndevices);
    return build_graph(n, m, row_ptr, col_idx, 0, out, false, &list, col_ptr, row_idx);
}

int qldpc_graph_create_host(int32_t n, int32_t m, const int32_t *row_ptr, const int32_t *col_idx,
                            qldpc_graph **out) {
    return build_graph(n, m, row_ptr, col_idx, 0, out, true);
}

int qldpc_graph_labels(const qldpc_graph *g, int32_t *labels_out, int64_t *stats_out) {
    if (!g) return fail(QLDPC_EINVAL, "graph is NULL");
    if (labels_out)
        for (int i = 0; i < g->n; ++i) labels_out[i] = g->col_lab.empty() ? i : g->col_lab[i];
    if (stats_out)
        for (int i = 0; i < 4; ++i) stats_out[i] = g->relabel_stats[i];
    return QLDPC_OK;
}

void qldpc_graph_destroy(qldpc_graph *g) {
    if (!g) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    for (auto &d : g->devs) {
        (void)hipSetDevice(d->device);
        (void)hipDeviceSynchronize();
        (void)hipFree(d->slot_meta);
        (void)hipFree(d->lane_row0);
        (void)hipFree(d->wave_rows);
        (void)hipFree(d->lane_head);
        (void)hipFree(d->lane_nst);
        (void)hipFree(d->slot_meta_ms);
        (void)hipFree(d->slot_meta2);
        (void)hipFree(d->slot_meta2_ms);
        (void)hipFree(d->hd_bits);
        (void)hipFree(d->hd_dv);
        (void)hipFree(d->stage_off);
        (void)hipFree(d->row_orig);
        (void)hipFree(d->part_row0);
        (void)hipFree(d->xoff);
        (void)hipFree(d->xbit);
        (void)hipFree(d->xbit_ms);
        (void)hipFree(d->vn_mask);
        (void)hipFree(d->vn_mask_ms);
        (void)hipFree(d->vn_exec);
        (void)hipFree(d->vn_exec_ms);
        (void)hipFree(d->lane_epl);
        (void)hipFree(d->ell_col);
        (void)hipFree(d->row_deg);
        (void)hipFree(d->iso_bits);
        (void)hipFree(d->vn_rows);
        (void)hipFree(d->vng_bits);
        (void)hipFree(d->vng_meta2);
        (void)hipFree(d->pair_src);
        (void)hipFree(d->pair_col);
        (void)hipFree(d->vng_rec);
        (void)hipFree(d->row_sem);
        (void)hipFree(d->row_rmask);
        (void)hipFree(d->col_orig);
        (void)hipFree(d->col_lab);
        (void)hipFree(d->ell_lab);
        for (auto &kv : d->ws) {
            (void)hipFree(kv.second.counter);
            (void)hipFree(kv.second.scratch);
            (void)hipFree(kv.second.codes);
            (void)hipFree(kv.second.palette);
            (void)hipFree(kv.second.pal_ok);
            (void)hipFree(kv.second.split_ctl);
            (void)hipFree(kv.second.llr_ws);
            if (kv.second.ev0) (void)hipEventDestroy(kv.second.ev0);
            if (kv.second.ev1) (void)hipEventDestroy(kv.second.ev1);
            (void)hipFree(kv.second.gtotal);
            (void)hipFree(kv.second.gstage);
        }
        for (auto &t : d->tslot) {
            (void)hipFree(t.seeds); (void)hipFree(t.clk); (void)hipFree(t.alice); (void)hipFree(t.bob);
            (void)hipFree(t.palice); (void)hipFree(t.pbob); (void)hipFree(t.alice_ext); (void)hipFree(t.synd);
            (void)hipFree(t.bits); (void)hipFree(t.ok); (void)hipFree(t.km); (void)hipFree(t.iters);
            (void)hipFree(t.tscratch); (void)hipFree(t.logp);
            (void)hipHostFree(t.h_iters); (void)hipHostFree(t.h_ok); (void)hipHostFree(t.h_km); (void)hipHostFree(t.h_clk);
            (void)hipHostFree(t.h_seeds); (void)hipHostFree(t.h_logp);
            for (hipEvent_t e : {t.ev0, t.ev_end[0], t.ev_end[1]})
                if (e) (void)hipEventDestroy(e);
            if (t.stream) (void)hipStreamDestroy(t.stream);
        }
        HostIO &io = d->io;
        (void)hipFree(io.llr); (void)hipFree(io.post); (void)hipFree(io.synd); (void)hipFree(io.bits); (void)hipFree(io.ok); (void)hipFree(io.iters);
        if (io.stream) (void)hipStreamDestroy(io.stream);
    }
    (void)hipSetDevice(prev);
    delete g;
}

int qldpc_graph_info(const qldpc_graph *g, int32_t *n, int32_t *m, int32_t *nnz, int32_t *num_devices) {
    if (!g) return fail(QLDPC_EINVAL, "graph is NULL");
    if (n) *n = g->n;
    if (m) *m = g->m;
    if (nnz) *nnz = g->E;
    if (num_devices) *num_devices = (int32_t)g->devs.size();
    return QLDPC_OK;
}

int qldpc_graph_plan(const qldpc_graph *g, int32_t device, int32_t algorithm, int32_t *lanes,
                     int32_t *edges_per_lane, int32_t *workgroups, int32_t *lds_bytes, const char **variant) {
    if (!g) return fail(QLDPC_EINVAL, "graph is NULL");
    if (algorithm < 0 || algorithm > 5) return fail(QLDPC_EINVAL, "algorithm must be 0..5");
    DeviceGraph *dg = find_dev(const_cast<qldpc_graph *>(g), device);
    // (a host-only graph answers everything but the device's workgroup count)
    if (!dg && !(g->devs.empty() && !workgroups)) return fail(QLDPC_EINVAL, "graph does not live on that device");
    const size_t lds = lds_of(*g, algorithm);
    // (split frames: the lanes that run — K parts of split_pl — not the arrays' stride)
    if (lanes) *lanes = (g->variant == VAR_V2 && g->split_k > 1) ? g->split_k * g->split_pl : g->T;
    if (edges_per_lane) *edges_per_lane = g->EPL;
    if (lds_bytes) *lds_bytes = (int32_t)lds;
    if (variant)
        *variant = (g->variant == VAR_V2 && g->split_k > 1) ? "v2_split"
                   : (g->variant == VAR_V2 && g->v2RG > 0) ? "v2_hybrid" : variant_name(g->variant);
    if (workgroups) {
        int prev = 0;
        HIP_TRY(hipGetDevice(&prev));
        HIP_TRY(hipSetDevice(dg->device));
        int b = 0;
        hipError_t e = g->variant == VAR_V2 ? occupancy_v2(g->v2R, g->v2RG, g->split_k, algorithm, block_threads(*g), lds, &b)
                                            : occupancy(g->variant, algorithm, g->T, lds, &b);
        (void)hipSetDevice(prev);
        if (e != hipSuccess) return hip_fail(e, "occupancy");
        *workgroups = b * dg->num_cus;
    }
    return QLDPC_OK;
}

int qldpc_graph_split_plan(const qldpc_graph *g, int32_t *parts, int32_t *part_lanes, int32_t *scratch_slots) {
    if (!g) return fail(QLDPC_EINVAL, "graph is NULL");
    const bool split = g->variant == VAR_V2 && g->split_k > 1;
    if (parts) *parts = split ? g->split_k : 1;
    if (part_lanes) *part_lanes = split ? g->split_pl : g->T;
    if (scratch_slots) *scratch_slots = g->variant == VAR_V2 ? g->v2RG : 0;
    return QLDPC_OK;
}

int qldpc_set_kernel_timing(qldpc_graph *g, int32_t enabled) {
    if (!g) return fail(QLDPC_EINVAL, "graph is NULL");
    g->kernel_timing = enabled != 0;
    return QLDPC_OK;
}

int qldpc_last_decode_kernel_ms(qldpc_graph *g, int32_t device, void *stream, float *ms) {
    if (!g || !ms) return fail(QLDPC_EINVAL, "graph / ms is NULL");
    DeviceGraph *dg = find_dev(g, device);
    if (!dg) return fail(QLDPC_EINVAL, "graph does not live on that device");
    hipEvent_t e0 = nullptr, e1 = nullptr;
    {
        std::lock_guard<std::mutex> lk(dg->mu);
        auto it = dg->ws.find(stream);
        if (it == dg->ws.end() || !it->second.ev_recorded)
            return fail(QLDPC_EINVAL, "no timed decode launch on that stream (qldpc_set_kernel_timing)");
        e0 = it->second.ev0;
        e1 = it->second.ev1;
    }
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(device));
    hipError_t e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(ms, e0, e1);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return hip_fail(e, "decode kernel events");
    return QLDPC_OK;
}

int qldpc_last_claim_order(qldpc_graph *g, int32_t device, void *stream, int32_t *order_out, int32_t *weight_out,
                           int32_t cap, int32_t *count) {
    if (!g || !count) return fail(QLDPC_EINVAL, "graph / count is NULL");
    DeviceGraph *dg = find_dev(g, device);
    if (!dg) return fail(QLDPC_EINVAL, "graph does not live on that device");
    // (the workspace lock is held across the wait and the copies: a decode on
    // the same stream with a larger batch would otherwise free and reallocate
    // forder / fweight under the copy)
    std::lock_guard<std::mutex> lk(dg->mu);
    auto it = dg->ws.find(stream);
    if (it == dg->ws.end()) return fail(QLDPC_EINVAL, "no decode on that stream");
    int32_t *const ord = it->second.forder, *const wt = it->second.fweight;
    const int cnt = it->second.order_count;
    *count = cnt;
    if (cnt == 0) return QLDPC_OK;
    if (cap < cnt) return fail(QLDPC_EINVAL, "order buffer smaller than the last batch");
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(device));
    hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e == hipSuccess && order_out) e = hipMemcpy(order_out, ord, (size_t)cnt * sizeof(int32_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess && weight_out) e = hipMemcpy(weight_out, wt, (size_t)cnt * sizeof(int32_t), hipMemcpyDeviceToHost);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return hip_fail(e, "claim order copy");
    return QLDPC_OK;
}

int qldpc_decode_batch_device(qldpc_graph *g, int32_t device, const qldpc_params *p, int32_t batch,
                              const double *d_llr, const uint8_t *d_syndrome, uint8_t *d_bits_out,
                              uint32_t *d_iters_out, uint8_t *d_synd_ok_out, double *d_posterior_out,
                              void *stream) {
    if (!g) return fail(QLDPC_EINVAL, "graph is NULL");
    int rc = check_params(p);
    if (rc) return rc;
    if (batch < 0) return fail(QLDPC_EINVAL, "batch must be >= 0");
    if (batch > 0 && (!d_llr || !d_syndrome || !d_bits_out || !d_iters_out || !d_synd_ok_out))
        return fail(QLDPC_EINVAL, "NULL device buffer");
    DeviceGraph *dg = find_dev(g, device);
    if (!dg) return fail(QLDPC_EINVAL, "graph does not live on that device");
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(device));
    rc = decode_on(g, dg, p, batch, d_llr, d_syndrome, d_bits_out, d_iters_out, d_synd_ok_out, d_posterior_out,
                   (hipStream_t)stream);
    (void)hipSetDevice(prev);
    return rc;
}

int qldpc_decode_batch(qldpc_graph *g, const qldpc_params *p, int32_t batch, const double *llr,
                       const uint8_t *syndrome, uint8_t *bits_out, uint32_t *iters_out, uint8_t *synd_ok_out,
                       double *posterior_out) {
    if (!g) return fail(QLDPC_EINVAL, "graph is NULL");
    int rc = check_params(p);
    if (rc) return rc;
    if (batch < 0) return fail(QLDPC_EINVAL, "batch must be >= 0");
    if (batch == 0) return QLDPC_OK;
    if (!llr || !syndrome || !bits_out || !iters_out || !synd_ok_out) return fail(QLDPC_EINVAL, "NULL host buffer");
    const int G = (int)g->devs.size();
    const int per = (batch + G - 1) / G;
    std::vector<int> rcs(G, QLDPC_OK);
    std::vector<std::string> errs(G);
    auto work = [&](int gi) {
        DeviceGraph *dg = g->devs[gi].get();
        const int f0 = gi * per, f1 = std::min(batch, f0 + per), nb = f1 - f0;
        if (nb <= 0) return;
        const size_t n = (size_t)g->n, m = (size_t)g->m;
        // One call at a time per device owns the staging buffers and their
        // stream, from the copy-in to the completed copy-out: concurrent host
        // threads on one shared graph (the reference's thread pool over
        // trials) serialise here instead of overwriting each other's frames.
        auto body = [&]() -> int {
            HIP_TRY(hipSetDevice(dg->device));
            std::lock_guard<std::mutex> io_lk(dg->io_mu);
            HostIO &io = dg->io;
            if (!io.stream) HIP_TRY(hipStreamCreateWithFlags(&io.stream, hipStreamNonBlocking));
            if ((size_t)nb > io.cap_frames) {
                int r;
                if ((r = grow(&io.llr, nb * n)) || (r = grow(&io.post, nb * n)) || (r = grow(&io.synd, nb * m)) ||
                    (r = grow(&io.bits, nb * n)) || (r = grow(&io.ok, (size_t)nb)) || (r = grow(&io.iters, (size_t)nb)))
                    return r;
                io.cap_frames = (size_t)nb;
            }
            HIP_TRY(hipMemcpyAsync(io.llr, llr + f0 * n, nb * n * sizeof(double), hipMemcpyHostToDevice, io.stream));
            HIP_TRY(hipMemcpyAsync(io.synd, syndrome + f0 * m, nb * m, hipMemcpyHostToDevice, io.stream));
            int r = decode_on(g, dg, p, nb, io.llr, io.synd, io.bits, io.iters, io.ok,
                              posterior_out ? io.post : nullptr, io.stream);
            if (r) {
                (void)hipStreamSynchronize(io.stream);  // nothing of this call stays in flight
                return r;
            }
            HIP_TRY(hipMemcpyAsync(bits_out + f0 * n, io.bits, nb * n, hipMemcpyDeviceToHost, io.stream));
            HIP_TRY(hipMemcpyAsync(iters_out + f0, io.iters, nb * sizeof(uint32_t), hipMemcpyDeviceToHost, io.stream));
            HIP_TRY(hipMemcpyAsync(synd_ok_out + f0, io.ok, nb, hipMemcpyDeviceToHost, io.stream));
            if (posterior_out)
                HIP_TRY(hipMemcpyAsync(posterior_out + f0 * n, io.post, nb * n * sizeof(double), hipMemcpyDeviceToHost,
                                       io.stream));
            HIP_TRY(hipStreamSynchronize(io.stream));
            return split_check(g, dg, io.stream);
        };
        const int r = body();
        rcs[gi] = r;
        if (r) errs[gi] = g_last_error;
    };
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    if (G == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int gi = 0; gi < G; ++gi) th.emplace_back(work, gi);
        for (auto &t : th) t.join();
    }
    (void)hipSetDevice(prev);
    for (int gi = 0; gi < G; ++gi)
        if (rcs[gi]) return fail(rcs[gi], errs[gi]);
    return QLDPC_OK;
}

int qldpc_build_frames_device(qldpc_graph *g, int32_t device, int32_t batch, const uint8_t *d_alice,
                              const uint8_t *d_bob, const double *d_log_p, double *d_llr, uint8_t *d_syndrome,
                              void *stream) {
    if (!g) return fail(QLDPC_EINVAL, "graph is NULL");
    if (batch < 0) return fail(QLDPC_EINVAL, "batch must be >= 0");
    if (batch > 0 && (!d_alice || !d_bob || !d_log_p || !d_llr || !d_syndrome))
        return fail(QLDPC_EINVAL, "NULL device buffer");
    DeviceGraph *dg = find_dev(g, device);
    if (!dg) return fail(QLDPC_EINVAL, "graph does not live on that device");
    if (int r = frame_builder_fits(g, -1)) return r;
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(device));
    hipError_t e = launch_build_frames(g->n, g->m, g->max_dc, dg->ell_col, dg->row_deg, batch, d_alice, d_bob,
                                       d_log_p, d_llr, d_syndrome, nullptr, nullptr, nullptr, nullptr,
                                       (hipStream_t)stream);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return hip_fail(e, "build_frames");
    return QLDPC_OK;
}

int qldpc_keys_match_device(int32_t batch, int32_t n, const uint8_t *d_alice, const uint8_t *d_bits,
                            uint8_t *d_keys_match, void *stream) {
    if (batch < 0 || n <= 0) return fail(QLDPC_EINVAL, "bad batch / n");
    if (batch > 0 && (!d_alice || !d_bits || !d_keys_match)) return fail(QLDPC_EINVAL, "NULL device buffer");
    hipError_t e = launch_keys_match(batch, n, d_alice, d_bits, d_keys_match, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "keys_match");
    return QLDPC_OK;
}

int qldpc_selftest_math_device(int32_t fn, int32_t count, const double *d_in, double *d_out, void *stream) {
    if (fn < 0 || fn > 9 || count < 0) return fail(QLDPC_EINVAL, "fn must be 0..9, count >= 0");
    if (count > 0 && (!d_in || !d_out)) return fail(QLDPC_EINVAL, "NULL device buffer");
    hipError_t e = launch_math_selftest(fn, count, d_in, d_out, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "math_selftest");
    return QLDPC_OK;
}

int qldpc_qkd_ldpc_batch_device(qldpc_graph *g, int32_t device, const qldpc_params *p, int32_t batch,
                                const uint8_t *d_alice, const uint8_t *d_bob, const double *d_log_p,
                                double *d_llr_ws, uint8_t *d_synd_ws, uint8_t *d_bits_out, uint32_t *d_iters_out,
                                uint8_t *d_synd_ok_out, uint8_t *d_keys_match_out, void *stream) {
    if (!g) return fail(QLDPC_EINVAL, "graph is NULL");
    int rc = check_params(p);
    if (rc) return rc;
    if (batch < 0) return fail(QLDPC_EINVAL, "batch must be >= 0");
    if (batch > 0 && (!d_alice || !d_bob || !d_log_p || !d_synd_ws || !d_bits_out || !d_iters_out || !d_synd_ok_out))
        return fail(QLDPC_EINVAL, "NULL device buffer");
    DeviceGraph *dg = find_dev(g, device);
    if (!dg) return fail(QLDPC_EINVAL, "graph does not live on that device");
    if (batch == 0) return QLDPC_OK;
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(device));
    rc = qkd_ldpc_window(g, dg, nullptr, p, batch, d_alice, d_bob, nullptr, nullptr, d_log_p, nullptr, d_llr_ws,
                         d_synd_ws, d_bits_out, d_iters_out, d_synd_ok_out, d_keys_match_out, (hipStream_t)stream);
    (void)hipSetDevice(prev);
    return rc;
}

// ---- rate adaptation (src/array_and_matrix_operations.cpp:1131-1223) ----------
int qldpc_xoshiro_state(uint64_t seed, uint64_t *state_out) {
    if (!state_out) return fail(QLDPC_EINVAL, "NULL state_out");
    Xoshiro256pp g(seed);
    for (int i = 0; i < 4; ++i) state_out[i] = g.s[i];
    return QLDPC_OK;
}

int qldpc_adapt_code_rate(int32_t n, int32_t m, double qber, double delta, double efficiency,
                          int32_t untainted_enabled, const int32_t *untainted, int32_t n_untainted,
                          uint64_t *prng_state, int32_t *punctured_out, int32_t *n_punctured, int32_t *shortened_out,
                          int32_t *n_shortened, double *adapted_rate_out) {
    if (n <= 0 || m < 0 || m >= n || !prng_state || !n_punctured || !n_shortened)
        return fail(QLDPC_EINVAL, "bad dimensions or NULL outputs");
    if (untainted_enabled && n_untainted > 0 && !untainted) return fail(QLDPC_EINVAL, "NULL untainted list");
    *n_punctured = 0;
    *n_shortened = 0;
    if (adapted_rate_out) *adapted_rate_out = 0.;
    Xoshiro256pp g(0);
    for (int i = 0; i < 4; ++i) g.s[i] = prng_state[i];
    const double h_b = -qber * std::log2(qber) - (1. - qber) * std::log2(1. - qber);
    const double optimal_R = 1. - efficiency * h_b;
    const double original_R = 1. - static_cast<double>(m) / static_cast<double>(n);
    const int num_short = static_cast<int>(std::ceil((original_R - optimal_R * (1. - delta)) * static_cast<double>(n)));
    const int num_punct = static_cast<int>(delta * static_cast<double>(n) - static_cast<double>(num_short));
    // beyond the achievable range: the reference warns and skips the combination
    if (num_short <= 0 || num_punct <= 0) return QLDPC_OK;
    std::vector<int> punct, bit_positions(n);
    if (untainted_enabled) {
        if (num_punct > n_untainted) return QLDPC_OK;
        punct.assign(untainted, untainted + num_punct);
    } else {
        for (int i = 0; i < n; ++i) bit_positions[i] = i;
        std::shuffle(bit_positions.begin(), bit_positions.end(), g);
        punct.assign(bit_positions.begin(), bit_positions.begin() + num_punct);
    }
    std::sort(punct.begin(), punct.end());
    for (int i = 0; i < n; ++i) bit_positions[i] = i;
    std::vector<int> remaining(n - num_punct);
    std::set_difference(bit_positions.begin(), bit_positions.end(), punct.begin(), punct.end(), remaining.begin());
    std::shuffle(remaining.begin(), remaining.end(), g);
    std::vector<int> shortened(remaining.begin(), remaining.begin() + num_short);
    std::sort(shortened.begin(), shortened.end());
    for (int i = 0; i < 4; ++i) prng_state[i] = g.s[i];
    *n_punctured = num_punct;
    *n_shortened = num_short;
    if (punctured_out) std::copy(punct.begin(), punct.end(), punctured_out);
    if (shortened_out) std::copy(shortened.begin(), shortened.end(), shortened_out);
    if (adapted_rate_out)
        *adapted_rate_out = static_cast<double>(n - m - num_short) / static_cast<double>(n - num_punct - num_short);
    return QLDPC_OK;
}

// ---- untainted puncturing (src/array_and_matrix_operations.cpp:975-1067) -----
// select_punctured_bits_untainted (arXiv:1103.6149): while untainted bits
// remain (X), take the bits of X with the fewest second-order neighbours
// (bits sharing a check, the bit itself excluded: get_second_order_neighbors,
// :975-996) inside X, in ascending order (std::set iteration), draw one with
// uniform_int_distribution<size_t>(0, candidates - 1) from the caller's
// generator, puncture it and remove it and its second-order neighbours from
// X.  Same candidates, same draws, same order as the reference's set-scanning
// loop; the counts |N2(i) n X| are kept incrementally instead of recounted
// (the relation is symmetric, so removing r decrements every q in N2(r)).
int qldpc_select_punctured_untainted(int32_t n, int32_t m, const int32_t *row_ptr, const int32_t *col_idx,
                                     const int32_t *col_ptr, const int32_t *row_idx, uint64_t *prng_state,
                                     int32_t *punctured_out, int32_t *n_punctured) {
    if (n <= 0 || m < 0 || !row_ptr || !col_idx || !col_ptr || !row_idx || !prng_state || !n_punctured)
        return fail(QLDPC_EINVAL, "bad dimensions or NULL arguments");
    *n_punctured = 0;
    if (row_ptr[m] != col_ptr[n]) return fail(QLDPC_EINVAL, "check_nodes / bit_nodes edge counts differ");
    for (int j = 0; j < m; ++j)
        for (int e = row_ptr[j]; e < row_ptr[j + 1]; ++e)
            if (col_idx[e] < 0 || col_idx[e] >= n) return fail(QLDPC_EINVAL, "bit index out of range");
    for (int i = 0; i < n; ++i)
        for (int e = col_ptr[i]; e < col_ptr[i + 1]; ++e)
            if (row_idx[e] < 0 || row_idx[e] >= m) return fail(QLDPC_EINVAL, "check index out of range");
    // N2(i): sorted, unique, without i
    std::vector<int64_t> n2p(n + 1, 0);
    std::vector<int32_t> n2;
    {
        std::vector<int32_t> tmp;
        for (int i = 0; i < n; ++i) {
            tmp.clear();
            for (int e = col_ptr[i]; e < col_ptr[i + 1]; ++e) {
                const int j = row_idx[e];
                tmp.insert(tmp.end(), col_idx + row_ptr[j], col_idx + row_ptr[j + 1]);
            }
            std::sort(tmp.begin(), tmp.end());
            tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
            for (int32_t b : tmp)
                if (b != i) n2.push_back(b);
            n2p[i + 1] = (int64_t)n2.size();
        }
    }
    Xoshiro256pp g(0);
    for (int i = 0; i < 4; ++i) g.s[i] = prng_state[i];
    std::vector<uint8_t> inx(n, 1);
    std::vector<int32_t> cnt(n), xs(n), cand, punct;
    for (int i = 0; i < n; ++i) cnt[i] = (int32_t)(n2p[i + 1] - n2p[i]);
    for (int i = 0; i < n; ++i) xs[i] = i;  // X in ascending order (compacted lazily)
    auto remove = [&](int r) {
        if (!inx[r]) return;
        inx[r] = 0;
        for (int64_t q = n2p[r]; q < n2p[r + 1]; ++q) --cnt[n2[q]];
    };
    while (!xs.empty()) {
        size_t w = 0;
        int32_t min_n = n;  // (the reference starts its minimum at num_bit_nodes)
        for (int32_t i : xs)
            if (inx[i]) {
                xs[w++] = i;
                if (cnt[i] < min_n) min_n = cnt[i];
            }
        xs.resize(w);
        if (xs.empty()) break;
        cand.clear();
        for (int32_t i : xs)
            if (cnt[i] == min_n) cand.push_back(i);
        std::uniform_int_distribution<size_t> d(0, cand.size() - 1);
        const int chosen = cand[d(g)];
        punct.push_back(chosen);
        remove(chosen);
        for (int64_t q = n2p[chosen]; q < n2p[chosen + 1]; ++q) remove(n2[q]);
    }
    for (int i = 0; i < 4; ++i) prng_state[i] = g.s[i];
    *n_punctured = (int32_t)punct.size();
    if (punctured_out) std::copy(punct.begin(), punct.end(), punctured_out);
    return QLDPC_OK;
}

int qldpc_rate_plan_create(qldpc_graph *g, int32_t n_punct, const int32_t *punctured, int32_t n_short,
                           const int32_t *shortened, qldpc_rate_plan **out) {
    if (!g || !out) return fail(QLDPC_EINVAL, "graph / out is NULL");
    *out = nullptr;
    if (n_punct < 0 || n_short < 0 || n_punct + n_short > g->n || (n_punct && !punctured) || (n_short && !shortened))
        return fail(QLDPC_EINVAL, "bad punctured / shortened lists");
    std::vector<uint8_t> cls(g->n, 0);
    std::vector<int32_t> src(g->n, 0);
    for (int i = 0; i < n_punct; ++i) {
        if (punctured[i] < 0 || punctured[i] >= g->n || (i && punctured[i] <= punctured[i - 1]))
            return fail(QLDPC_EINVAL, "punctured positions must be ascending and in [0, n)");
        cls[punctured[i]] = 1;
        src[punctured[i]] = i;
    }
    for (int i = 0; i < n_short; ++i) {
        if (shortened[i] < 0 || shortened[i] >= g->n || (i && shortened[i] <= shortened[i - 1]))
            return fail(QLDPC_EINVAL, "shortened positions must be ascending and in [0, n)");
        if (cls[shortened[i]]) return fail(QLDPC_EINVAL, "a position is both punctured and shortened");
        cls[shortened[i]] = 2;
    }
    int key = 0;
    for (int i = 0; i < g->n; ++i)
        if (cls[i] == 0) src[i] = key++;
    auto plan = std::make_unique<qldpc_rate_plan>();
    plan->n_punct = n_punct;
    plan->n_short = n_short;
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    for (auto &dg : g->devs) {
        HIP_TRY(hipSetDevice(dg->device));
        uint8_t *dc = nullptr;
        int32_t *ds = nullptr;
        int rc;
        if ((rc = upload(&dc, cls)) || (rc = upload(&ds, src))) {
            (void)hipSetDevice(prev);
            return rc;
        }
        plan->devs.push_back({dg->device, dc, ds});
    }
    HIP_TRY(hipSetDevice(prev));
    *out = plan.release();
    return QLDPC_OK;
}

void qldpc_rate_plan_destroy(qldpc_rate_plan *plan) {
    if (!plan) return;
    for (auto &d : plan->devs) {
        (void)hipFree(d.cls);
        (void)hipFree(d.src);
    }
    delete plan;
}

namespace {
// The generator workspace of the _device entries, one per (device, stream),
// kept across calls so a stream-pipelined caller's launches stay asynchronous
// (grown, never shrunk; growing drains the device before freeing the old one).
std::mutex g_tws_mu;
std::map<std::pair<int, hipStream_t>, std::pair<uint32_t *, size_t>> g_tws;
hipError_t trial_workspace(hipStream_t s, size_t words, uint32_t **out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_tws_mu);
    auto &w = g_tws[{dev, s}];
    if (w.second < words) {
        if (w.first) {
            if ((e = hipDeviceSynchronize()) != hipSuccess) return e;
            (void)hipFree(w.first);
            w = {nullptr, 0};
        }
        if ((e = hipMalloc(&w.first, std::max<size_t>(words, 1) * sizeof(uint32_t))) != hipSuccess) return e;
        w.second = words;
    }
    *out = w.first;
    return hipSuccess;
}
}  // namespace

int qldpc_trials_rate_adapt_device(int32_t n, double qber, int32_t batch, const uint64_t *d_seeds, uint64_t seed_add,
                                   int32_t n_punct, uint8_t *d_alice, uint8_t *d_bob, uint8_t *d_punct_alice,
                                   uint8_t *d_punct_bob, double *accurate_qber_out, void *stream) {
    if (n_punct < 0 || (n_punct > 0 && batch > 0 && (!d_punct_alice || !d_punct_bob)))
        return fail(QLDPC_EINVAL, "bad n_punct / NULL punctured-draw buffers");
    if (n <= 0 || batch < 0) return fail(QLDPC_EINVAL, "n must be > 0 and batch >= 0");
    const uint64_t n_err = (uint64_t)((double)n * qber);
    if (n_err == 0) return fail(QLDPC_EINVAL, "Key size '" + std::to_string(n) + "' is too small for QBER.");
    if (n_err > (uint64_t)n) return fail(QLDPC_EINVAL, "QBER must be <= 1");
    if (accurate_qber_out) *accurate_qber_out = (double)n_err / (double)n;
    if (batch == 0) return QLDPC_OK;
    if (!d_seeds || !d_alice || !d_bob) return fail(QLDPC_EINVAL, "NULL device buffer");
    const hipStream_t s = (hipStream_t)stream;
    uint32_t *scratch = nullptr;
    HIP_TRY(trial_workspace(s, trials_scratch_words(n, n_err, n_punct, batch), &scratch));
    hipError_t e = launch_trials(n, n_err, batch, d_seeds, seed_add, d_alice, d_bob, scratch, n_punct, d_punct_alice,
                                 d_punct_bob, s);
    if (e != hipSuccess) return hip_fail(e, "trials_rate_adapt");
    return QLDPC_OK;
}

int qldpc_build_frames_rate_adapt_device(qldpc_graph *g, const qldpc_rate_plan *plan, int32_t device, int32_t batch,
                                         const uint8_t *d_alice, const uint8_t *d_bob, const uint8_t *d_punct_alice,
                                         const uint8_t *d_punct_bob, const double *d_log_p, uint8_t *d_alice_ext,
                                         double *d_llr, uint8_t *d_syndrome, void *stream) {
    if (!g || !plan) return fail(QLDPC_EINVAL, "graph / plan is NULL");
    if (batch < 0) return fail(QLDPC_EINVAL, "batch must be >= 0");
    if (batch > 0 && (!d_alice || !d_bob || !d_log_p || !d_alice_ext || !d_llr || !d_syndrome ||
                      (plan->n_punct && (!d_punct_alice || !d_punct_bob))))
        return fail(QLDPC_EINVAL, "NULL device buffer");
    DeviceGraph *dg = find_dev(g, device);
    const qldpc_rate_plan::Dev *pd = nullptr;
    for (auto &d : plan->devs)
        if (d.device == device) pd = &d;
    if (!dg || !pd) return fail(QLDPC_EINVAL, "graph / plan does not live on that device");
    if (int r = frame_builder_fits(g, plan->n_punct)) return r;
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(device));
    hipError_t e = launch_build_frames_ra(g->n, g->m, dg->ell_col, dg->row_deg, pd->cls, pd->src, plan->n_punct, batch,
                                          d_alice, d_bob, d_punct_alice, d_punct_bob, d_log_p, d_alice_ext, d_llr,
                                          d_syndrome, nullptr, nullptr, nullptr, nullptr, (hipStream_t)stream);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return hip_fail(e, "build_frames_rate_adapt");
    return QLDPC_OK;
}

int qldpc_qkd_ldpc_rate_adapt_batch_device(qldpc_graph *g, const qldpc_rate_plan *plan, int32_t device,
                                           const qldpc_params *p, int32_t batch, const uint8_t *d_alice,
                                           const uint8_t *d_bob, const uint8_t *d_punct_alice,
                                           const uint8_t *d_punct_bob, const double *d_log_p, uint8_t *d_alice_ext,
                                           double *d_llr_ws, uint8_t *d_synd_ws, uint8_t *d_bits_out,
                                           uint32_t *d_iters_out, uint8_t *d_synd_ok_out, uint8_t *d_keys_match_out,
                                           void *stream) {
    if (!g || !plan) return fail(QLDPC_EINVAL, "graph / plan is NULL");
    int rc = check_params(p);
    if (rc) return rc;
    if (batch < 0) return fail(QLDPC_EINVAL, "batch must be >= 0");
    if (batch == 0) return QLDPC_OK;
    if (!d_alice || !d_bob || !d_log_p || !d_alice_ext || !d_synd_ws || !d_bits_out || !d_iters_out ||
        !d_synd_ok_out || (plan->n_punct && (!d_punct_alice || !d_punct_bob)))
        return fail(QLDPC_EINVAL, "NULL device buffer");
    DeviceGraph *dg = find_dev(g, device);
    if (!dg) return fail(QLDPC_EINVAL, "graph does not live on that device");
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(device));
    rc = qkd_ldpc_window(g, dg, plan, p, batch, d_alice, d_bob, d_punct_alice, d_punct_bob, d_log_p, d_alice_ext,
                         d_llr_ws, d_synd_ws, d_bits_out, d_iters_out, d_synd_ok_out, d_keys_match_out,
                         (hipStream_t)stream);
    (void)hipSetDevice(prev);
    return rc;
}

// ---- simulation-driver helpers (src/config.cpp, src/array_and_matrix_operations.cpp:121-256) ----
int qldpc_sort_permutation(const double *keys, int32_t n, int32_t *perm_out) {
    if (n < 0 || (n > 0 && (!keys || !perm_out))) return fail(QLDPC_EINVAL, "bad n / NULL arrays");
    // The reference sorts config structs by code_rate with std::sort (not
    // stable): the same libstdc++ algorithm on the same key sequence moves the
    // elements identically, so the permutation of (key, index) pairs is theirs.
    std::vector<std::pair<double, int32_t>> v(n);
    for (int32_t i = 0; i < n; ++i) v[i] = {keys[i], i};
    std::sort(v.begin(), v.end(), [](const std::pair<double, int32_t> &a, const std::pair<double, int32_t> &b) {
        return a.first < b.first;
    });
    for (int32_t i = 0; i < n; ++i) perm_out[i] = v[i].second;
    return QLDPC_OK;
}

int qldpc_bits_to_remove(int32_t n, int32_t m, const int32_t *col_ptr, const int32_t *row_idx, int32_t n_punct,
                         const int32_t *punctured, int32_t n_short, const int32_t *shortened, int32_t rate_adapt,
                         int32_t *out, int32_t *count) {
    if (n <= 0 || m < 0 || !col_ptr || !row_idx || !count || (n_punct && !punctured) || (n_short && !shortened))
        return fail(QLDPC_EINVAL, "bad arguments");
    // find_available_index over a marked-check bitmap (same first-unmarked choice
    // as std::find over the marked list, in O(E) overall).
    std::vector<char> marked(m, 0);
    auto take = [&](int i) -> bool {
        for (int e = col_ptr[i]; e < col_ptr[i + 1]; ++e)
            if (!marked[row_idx[e]]) {
                marked[row_idx[e]] = 1;
                return true;
            }
        return false;
    };
    std::vector<int> removed;
    std::vector<std::pair<int, int>> cand;  // (bit, column weight)
    if (rate_adapt) {  // get_bits_positions_to_remove_rate_adapt (:189-256)
        int s = 0, p = 0;
        for (int i = 0; i < n; ++i) {
            if (s < n_short && shortened[s] == i) {
                removed.push_back(i);
                ++s;
            } else if (p < n_punct && punctured[p] == i) {
                removed.push_back(i);
                take(i);
                ++p;
            } else {
                cand.push_back({i, col_ptr[i + 1] - col_ptr[i]});
            }
        }
    } else {  // get_bits_positions_to_remove (:138-185)
        for (int i = 0; i < n; ++i) cand.push_back({i, col_ptr[i + 1] - col_ptr[i]});
    }
    // std::sort by column weight (not stable): same algorithm, same order as the reference
    std::sort(cand.begin(), cand.end(),
              [](const std::pair<int, int> &a, const std::pair<int, int> &b) { return a.second < b.second; });
    for (const auto &c : cand)
        if (take(c.first)) removed.push_back(c.first);
    std::sort(removed.begin(), removed.end());
    *count = (int32_t)removed.size();
    if (out) std::copy(removed.begin(), removed.end(), out);
    return QLDPC_OK;
}

// ---- trial generator (src/simulation.cpp:540-551,713-719,743) ----------------
int qldpc_trial_seeds(uint64_t simulation_seed, int32_t count, uint64_t *seeds_out) {
    if (count < 0 || (count > 0 && !seeds_out)) return fail(QLDPC_EINVAL, "bad count / NULL seeds_out");
    // The reference draws seeds with uniform_int_distribution<size_t>(0,
    // SIZE_MAX), which passes each 64-bit output through unchanged.
    Xoshiro256pp g(simulation_seed);
    std::uniform_int_distribution<size_t> d(0, std::numeric_limits<size_t>::max());
    for (int32_t i = 0; i < count; ++i) seeds_out[i] = d(g);
    return QLDPC_OK;
}

int qldpc_xoshiro_jump(uint64_t seed, uint64_t draws, uint64_t *state_out) {
    if (!state_out) return fail(QLDPC_EINVAL, "NULL state_out");
    return xoshiro_jump_check(seed, draws, state_out);
}

int qldpc_trials_device(int32_t n, double qber, int32_t batch, const uint64_t *d_seeds, uint64_t seed_add,
                        uint8_t *d_alice, uint8_t *d_bob, double *accurate_qber_out, void *stream) {
    if (n <= 0 || batch < 0) return fail(QLDPC_EINVAL, "n must be > 0 and batch >= 0");
    const uint64_t n_err = (uint64_t)((double)n * qber);
    if (n_err == 0)  // run_trial's own check (src/simulation.cpp:552-553)
        return fail(QLDPC_EINVAL, "Key size '" + std::to_string(n) + "' is too small for QBER.");
    if (n_err > (uint64_t)n) return fail(QLDPC_EINVAL, "QBER must be <= 1");
    if (accurate_qber_out) *accurate_qber_out = (double)n_err / (double)n;
    if (batch == 0) return QLDPC_OK;
    if (!d_seeds || !d_alice || !d_bob) return fail(QLDPC_EINVAL, "NULL device buffer");
    const hipStream_t s = (hipStream_t)stream;
    uint32_t *scratch = nullptr;
    HIP_TRY(trial_workspace(s, trials_scratch_words(n, n_err, 0, batch), &scratch));
    hipError_t e = launch_trials(n, n_err, batch, d_seeds, seed_add, d_alice, d_bob, scratch, 0, nullptr, nullptr, s);
    if (e != hipSuccess) return hip_fail(e, "trials");
    return QLDPC_OK;
}


// ---- the batch seam of the simulation loop (src/simulation.cpp:721-746) ------
int qldpc_shard_range(int32_t count, int32_t shards, int32_t shard, int32_t *lo, int32_t *hi) {
    if (count < 0 || shards <= 0 || shard < 0 || shard >= shards || !lo || !hi)
        return fail(QLDPC_EINVAL, "bad count / shards / shard / NULL bounds");
    // contiguous slices of ceil(count / shards); trailing shards may be short or empty
    const int64_t per = ((int64_t)count + shards - 1) / shards;
    *lo = (int32_t)std::min<int64_t>(count, (int64_t)shard * per);
    *hi = (int32_t)std::min<int64_t>(count, (int64_t)*lo + per);
    return QLDPC_OK;
}

// One combination's trials in flight: where its results go, and the first
// error of each device's slice.  Its chunks sit in the devices' pipeline slots
// (TrialSlot::owner) until harvested — by qldpc_run_trials_wait, or by a later
// submit that needs the slot.
struct qldpc_trials_job {
    qldpc_graph *g = nullptr;
    uint32_t *iters_out = nullptr;
    uint8_t *synd_ok_out = nullptr, *keys_match_out = nullptr;
    double *runtime_us_out = nullptr;
    std::vector<int> rcs;           // per device slice (written under that device's trial_mu)
    std::vector<std::string> errs;
};

namespace {

// Wait for a slot's chunk and deliver its results to the job that owns it:
// per trial {iterations, syndromes_match, keys_match} and its share of the
// chunk's window (QKD_LDPC's per-trial window on device, HIP events on the
// slot's stream) in proportion to its own decode span.  dg->trial_mu held.
int harvest_slot(qldpc_graph *g, DeviceGraph *dg, int gi, TrialSlot &t) {
    if (t.nb == 0) return QLDPC_OK;
    qldpc_trials_job *job = t.owner;
    const int nb = t.nb;
    t.nb = 0;
    t.owner = nullptr;
    auto body = [&]() -> int {
        HIP_TRY(hipStreamSynchronize(t.stream));
        int r = split_check(g, dg, t.stream);
        if (r) return r;
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, t.ev0, t.ev1));
        if (t.prev_end) {  // (ended before this chunk's decode began: the stream waited for it)
            float mp = 0.f;
            HIP_TRY(hipEventElapsedTime(&mp, t.prev_end, t.ev1));
            if (mp < ms) ms = mp;
            t.prev_end = nullptr;
        }
        double span_sum = 0.;
        for (int i = 0; i < nb; ++i) span_sum += (double)(t.h_clk[2 * i + 1] - t.h_clk[2 * i]);
        for (int i = 0; i < nb; ++i) {
            job->iters_out[t.f0 + i] = t.h_iters[i];
            job->synd_ok_out[t.f0 + i] = t.h_ok[i];
            job->keys_match_out[t.f0 + i] = t.h_km[i];
            if (job->runtime_us_out) {
                const double span = (double)(t.h_clk[2 * i + 1] - t.h_clk[2 * i]);
                job->runtime_us_out[t.f0 + i] =
                    span_sum > 0. ? 1e3 * (double)ms * span / span_sum : 1e3 * (double)ms / nb;
            }
        }
        return QLDPC_OK;
    };
    const int r = body();
    if (r && job->rcs[gi] == QLDPC_OK) {  // the error belongs to the owning job's slice
        job->rcs[gi] = r;
        job->errs[gi] = g_last_error;
    }
    return r;
}

}  // namespace

int qldpc_run_trials_submit(qldpc_graph *g, const qldpc_rate_plan *plan, const qldpc_params *p, double qber,
                            int32_t count, const uint64_t *seeds, uint64_t seed_add, uint32_t *iters_out,
                            uint8_t *synd_ok_out, uint8_t *keys_match_out, double *runtime_us_out,
                            double *accurate_qber_out, qldpc_trials_job **job_out) {
    if (!job_out) return fail(QLDPC_EINVAL, "job_out is NULL");
    *job_out = nullptr;
    if (!g) return fail(QLDPC_EINVAL, "graph is NULL");
    int rc = check_params(p);
    if (rc) return rc;
    if (count < 0) return fail(QLDPC_EINVAL, "count must be >= 0");
    if (g->devs.empty()) return fail(QLDPC_EINVAL, "graph has no device (host-only)");
    const int n = g->n;
    const uint64_t n_err = (uint64_t)((double)n * qber);
    if (n_err == 0)  // run_trial's own check (src/simulation.cpp:552-553)
        return fail(QLDPC_EINVAL, "Key size '" + std::to_string(n) + "' is too small for QBER.");
    if (n_err > (uint64_t)n) return fail(QLDPC_EINVAL, "QBER must be <= 1");
    const double q_acc = (double)n_err / (double)n;  // inject_errors' return (:922-933)
    if (accurate_qber_out) *accurate_qber_out = q_acc;
    if (count > 0 && (!seeds || !iters_out || !synd_ok_out || !keys_match_out))
        return fail(QLDPC_EINVAL, "NULL host buffer");
    if (plan && plan->n_punct + plan->n_short > n) return fail(QLDPC_EINVAL, "rate plan does not fit the graph");
    const int G = (int)g->devs.size();
    std::unique_ptr<qldpc_trials_job> job(new qldpc_trials_job);
    job->g = g;
    job->iters_out = iters_out;
    job->synd_ok_out = synd_ok_out;
    job->keys_match_out = keys_match_out;
    job->runtime_us_out = runtime_us_out;
    job->rcs.assign(G, QLDPC_OK);
    job->errs.assign(G, std::string());
    if (count == 0) {
        *job_out = job.release();
        return QLDPC_OK;
    }
    const double lp = qldpc_log_p(q_acc);  // log((1 - q) / q) by the host C library (:1043)
    const int n_punct = plan ? plan->n_punct : 0;
    // Bytes of one trial in a pipeline slot (keys, frames, results, generator workspace).
    const size_t per_frame = 4 * (size_t)n + (size_t)g->m + 2 * (size_t)n_punct + 64 +
                             4 * trials_scratch_words(n, n_err, n_punct, 64) / 64;
    // Frames per chunk: a device's whole slice within ~512 MiB of the slot's own
    // buffers (16384 frames at most); longer slices alternate chunks over the
    // two slots.  (The persistent decode holds every CU, so halving a slice buys
    // no overlap: C2, 4096 trials, 2 x 2048 took 22.3 ms, 1 x 4096 21.5 ms;
    // profiles/r04/seam_chunk_ab.txt.)  QLDPC_TRIAL_CHUNK overrides.
    int cap = (int)std::max<size_t>(1, std::min<size_t>(16384, ((size_t)512 << 20) / per_frame));
    if (env_int("QLDPC_TRIAL_CHUNK", 0) > 0) cap = env_int("QLDPC_TRIAL_CHUNK", 0);
    qldpc_trials_job *J = job.get();
    auto work = [&](int gi) {
        DeviceGraph *dg = g->devs[gi].get();
        int32_t lo = 0, hi = 0;
        (void)qldpc_shard_range(count, G, gi, &lo, &hi);
        if (hi <= lo) return;
        auto body = [&]() -> int {
            HIP_TRY(hipSetDevice(dg->device));
            std::lock_guard<std::mutex> lk(dg->trial_mu);
            auto ensure = [&](TrialSlot &t, int nb) -> int {
                if (!t.stream) HIP_TRY(hipStreamCreateWithFlags(&t.stream, hipStreamNonBlocking));
                if (!t.ev0) HIP_TRY(hipEventCreate(&t.ev0));
                for (hipEvent_t &e : t.ev_end)
                    if (!e) HIP_TRY(hipEventCreate(&e));
                if ((size_t)nb > t.cap || (size_t)std::max(n_punct, 1) > t.cap_punct) {
                    const size_t c = std::max((size_t)nb, t.cap), cp = std::max((size_t)std::max(n_punct, 1), t.cap_punct);
                    int r;
                    if ((r = grow(&t.seeds, c)) || (r = grow(&t.clk, 2 * c)) || (r = grow(&t.alice, c * n)) ||
                        (r = grow(&t.bob, c * n)) || (r = grow(&t.alice_ext, c * n)) || (r = grow(&t.bits, c * n)) ||
                        (r = grow(&t.synd, c * (size_t)std::max(g->m, 1))) || (r = grow(&t.ok, c)) ||
                        (r = grow(&t.km, c)) || (r = grow(&t.iters, c)) || (r = grow(&t.logp, c)) ||
                        (r = grow(&t.palice, c * cp)) || (r = grow(&t.pbob, c * cp)))
                        return r;

                    (void)hipHostFree(t.h_iters); (void)hipHostFree(t.h_ok); (void)hipHostFree(t.h_km); (void)hipHostFree(t.h_clk);
                    (void)hipHostFree(t.h_seeds); (void)hipHostFree(t.h_logp);
                    t.h_iters = nullptr; t.h_ok = nullptr; t.h_km = nullptr; t.h_clk = nullptr; t.cap = 0;
                    t.h_seeds = nullptr; t.h_logp = nullptr;
                    HIP_TRY(hipHostMalloc(&t.h_iters, c * sizeof(uint32_t)));
                    HIP_TRY(hipHostMalloc(&t.h_ok, c));
                    HIP_TRY(hipHostMalloc(&t.h_km, c));
                    HIP_TRY(hipHostMalloc(&t.h_clk, 2 * c * sizeof(uint64_t)));
                    HIP_TRY(hipHostMalloc(&t.h_seeds, c * sizeof(uint64_t)));
                    HIP_TRY(hipHostMalloc(&t.h_logp, c * sizeof(double)));
                    t.cap = c;
                    t.cap_punct = cp;
                }
                // the generator's workspace also grows with the error count k
                const size_t sw = trials_scratch_words(n, n_err, n_punct, (int)t.cap);
                if (sw > t.tscratch_words) {
                    int r = grow(&t.tscratch, sw);
                    if (r) return r;
                    t.tscratch_words = sw;
                }
                return QLDPC_OK;
            };
            int r = QLDPC_OK;
            for (int f = lo; f < hi && !r;) {
                TrialSlot &t = dg->tslot[dg->next_slot];
                dg->next_slot ^= 1;
                const TrialSlot &o = dg->tslot[dg->next_slot];  // the other slot
                (void)harvest_slot(g, dg, gi, t);  // (a previous chunk, possibly another job's)
                const int nb = std::min(cap, hi - f);
                if ((r = ensure(t, nb))) break;
                auto enqueue = [&]() -> int {
                    // (the slot's pinned inputs are free: its previous chunk was harvested)
                    std::memcpy(t.h_seeds, seeds + f, (size_t)nb * sizeof(uint64_t));
                    std::fill(t.h_logp, t.h_logp + nb, lp);
                    HIP_TRY(hipMemcpyAsync(t.seeds, t.h_seeds, (size_t)nb * sizeof(uint64_t), hipMemcpyHostToDevice,
                                           t.stream));
                    HIP_TRY(hipMemcpyAsync(t.logp, t.h_logp, (size_t)nb * sizeof(double), hipMemcpyHostToDevice,
                                           t.stream));
                    // run_trial's keys (+ QKD_LDPC_RATE_ADAPT's punctured draws), seed = seeds[n] + curr_sim (:743)
                    HIP_TRY(launch_trials(n, n_err, nb, t.seeds, seed_add, t.alice, t.bob, t.tscratch, n_punct,
                                          t.palice, t.pbob, t.stream));
                    // Trial generation, frame build and claim order overlap the
                    // other slot's chunk (the previous chunk, or the previous
                    // combination's under qldpc_run_trials_submit); the decode
                    // waits for it to end, so two decodes never share the CUs
                    // and the chunk's window, started no earlier than that end
                    // (harvest_slot), is its own work.
                    HIP_TRY(hipEventRecord(t.ev0, t.stream));
                    t.ev_i ^= 1;
                    t.ev1 = t.ev_end[t.ev_i];
                    t.prev_end = o.nb > 0 ? o.ev1 : nullptr;
                    int rr = qkd_ldpc_window(g, dg, plan, p, nb, t.alice, t.bob, t.palice, t.pbob, t.logp, t.alice_ext,
                                             nullptr, t.synd, t.bits, t.iters, t.ok, t.km, t.stream, t.clk,
                                             t.prev_end);
                    if (rr) return rr;
                    HIP_TRY(hipEventRecord(t.ev1, t.stream));
                    HIP_TRY(hipMemcpyAsync(t.h_iters, t.iters, (size_t)nb * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                           t.stream));
                    HIP_TRY(hipMemcpyAsync(t.h_ok, t.ok, (size_t)nb, hipMemcpyDeviceToHost, t.stream));
                    HIP_TRY(hipMemcpyAsync(t.h_km, t.km, (size_t)nb, hipMemcpyDeviceToHost, t.stream));
                    HIP_TRY(hipMemcpyAsync(t.h_clk, t.clk, 2 * (size_t)nb * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                           t.stream));
                    return QLDPC_OK;
                };
                if ((r = enqueue())) {
                    (void)hipStreamSynchronize(t.stream);  // nothing of this chunk stays in flight
                    break;
                }
                t.owner = J;
                t.f0 = f;
                t.nb = nb;
                f += nb;
            }
            if (r) {  // an error: drain this job's chunks in flight on the device
                for (auto &t : dg->tslot)
                    if (t.owner == J) {
                        (void)hipStreamSynchronize(t.stream);
                        t.nb = 0;
                        t.owner = nullptr;
                    }
            }
            return r;
        };
        const int r = body();
        if (r) {
            std::lock_guard<std::mutex> lk(dg->trial_mu);
            if (J->rcs[gi] == QLDPC_OK) {
                J->rcs[gi] = r;
                J->errs[gi] = g_last_error;
            }
        }
    };
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    if (G == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int gi = 0; gi < G; ++gi) th.emplace_back(work, gi);
        for (auto &t : th) t.join();
    }
    (void)hipSetDevice(prev);
    *job_out = job.release();
    return QLDPC_OK;
}

int qldpc_run_trials_wait(qldpc_trials_job *job) {
    if (!job) return fail(QLDPC_EINVAL, "job is NULL");
    std::unique_ptr<qldpc_trials_job> own(job);
    qldpc_graph *g = job->g;
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    for (int gi = 0; gi < (int)g->devs.size(); ++gi) {
        DeviceGraph *dg = g->devs[gi].get();
        std::lock_guard<std::mutex> lk(dg->trial_mu);
        if (hipSetDevice(dg->device) != hipSuccess) continue;
        for (auto &t : dg->tslot)
            if (t.owner == job) (void)harvest_slot(g, dg, gi, t);
    }
    (void)hipSetDevice(prev);
    for (int gi = 0; gi < (int)job->rcs.size(); ++gi)
        if (job->rcs[gi]) return fail(job->rcs[gi], job->errs[gi]);
    return QLDPC_OK;
}

int qldpc_run_trials(qldpc_graph *g, const qldpc_rate_plan *plan, const qldpc_params *p, double qber, int32_t count,
                     const uint64_t *seeds, uint64_t seed_add, uint32_t *iters_out, uint8_t *synd_ok_out,
                     uint8_t *keys_match_out, double *runtime_us_out, double *accurate_qber_out) {
    qldpc_trials_job *job = nullptr;
    const int rc = qldpc_run_trials_submit(g, plan, p, qber, count, seeds, seed_add, iters_out, synd_ok_out,
                                           keys_match_out, runtime_us_out, accurate_qber_out, &job);
    if (rc) return rc;
    return qldpc_run_trials_wait(job);
}

}  // extern "C"
