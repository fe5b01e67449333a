// decoder.hip — gfx950 flooding belief-propagation decoder for QKD-LDPC.
//
// Hot path of ColdCloudd/QKD_LDPC_V: the six decoders of
// src/qkd_ldpc_algorithm.cpp:3-1029 (SPA :3-144, SPA-linear :174-315,
// NMSA :317-482, OMSA :484-650, ANMSA :652-839, AOMSA :841-1029), batched over
// independent frames.  Results are bit-identical to the reference: same IEEE
// operation sequence per message (no FMA contraction: built with
// -ffp-contract=off), glibc-exact tanh/atanh (exact_math.h), the reference's
// row-order products and std::accumulate-order sums.
//
// Mapping to the machine:
//   * one workgroup decodes one frame at a time; workgroups are persistent and
//     pull frame ids from a device counter, so an early-exiting frame frees its
//     CU at once (frames converge after 3..50 iterations);
//   * the frame's E edges are dealt to the T lanes in CSR (row-major) order,
//     EPL consecutive edges per lane; the lane keeps those edges' messages in
//     VGPRs across iterations (variant REG_LDS) or in a coalesced slot-major
//     per-workgroup scratch (GLB_*);
//   * posterior totals live in LDS (REG_LDS, GLB_LDS): every gather of a bit's
//     total is an LDS read, never a scattered HBM read;
//   * a row may straddle two lanes: its sequential product (SPA) or min1/min2
//     aggregate (min-sum) is carried across the boundary through LDS;
//   * variable-node sums are accumulated in the reference's order
//     ((llr + c0) + c1) + ... by dv_max phases: phase k adds the message of every
//     edge that is the k-th edge of its bit.
#include <float.h>

#include <map>
#include <mutex>

#include "decoder_common.hpp"

namespace qldpc {

namespace {

using namespace dev;

constexpr int CTRL_BYTES = 16;


__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// Byte layout of the per-frame state block (LDS or global scratch).
struct FrameLayout {
    size_t total, rowA, rowB, carryA, carryB, carryI, rowflag, bytes;
    __host__ __device__ FrameLayout(int n, int m, int T) {
        size_t o = 0;
        total = o; o = align16(o + (size_t)n * 8);
        rowA = o; o = align16(o + (size_t)m * 8);
        rowB = o; o = align16(o + (size_t)m * 8);
        carryA = o; o = align16(o + (size_t)T * 8);
        carryB = o; o = align16(o + (size_t)T * 8);
        carryI = o; o = align16(o + (size_t)T * 4);
        rowflag = o; o = align16(o + (size_t)m);
        bytes = o;
    }
};

template <int ALG, int R, bool TOT_LDS>
__global__ void __launch_bounds__(1024) decode_kernel(DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool SPA_FAM = (ALG == 0 || ALG == 1);
    constexpr bool ADAPT = (ALG == 4 || ALG == 5);
    constexpr bool NORM = (ALG == 2 || ALG == 4);

    const int tid = threadIdx.x;
    const int T = a.T, n = a.n, m = a.m, EPL = a.EPL;
    const double thr = a.thr;
    const bool thr_on = a.thr_on != 0;

    double *wg = a.scratch ? a.scratch + (size_t)blockIdx.x * (size_t)a.scratch_wg_doubles : nullptr;
    const FrameLayout L(n, m, T);
    unsigned char *fb;
    if constexpr (TOT_LDS) fb = smem + CTRL_BYTES;
    else fb = reinterpret_cast<unsigned char *>(wg + (R == 0 ? (size_t)EPL * T : 0));
    double *total = reinterpret_cast<double *>(fb + L.total);
    double *rowA = reinterpret_cast<double *>(fb + L.rowA);
    double *rowB = reinterpret_cast<double *>(fb + L.rowB);
    double *carryA = reinterpret_cast<double *>(fb + L.carryA);
    double *carryB = reinterpret_cast<double *>(fb + L.carryB);
    int *carryI = reinterpret_cast<int *>(fb + L.carryI);
    uint8_t *rowflag = fb + L.rowflag;  // bit0 target syndrome, bit1 row mismatch, bit2 neg parity
    int *s_frame = reinterpret_cast<int *>(smem);

    EdgeMsgs<R> c2b;
    if constexpr (R == 0) c2b.bind(wg, tid, T);
    // occurrence pairing (unsorted adjacency): global-slot instantiations only
    double *const pbuf = (R == 0 && a.pair_src) ? wg + a.pair_buf_off : nullptr;

    MetaSrc<R> meta;
    meta.init(a.slot_meta, tid, T);
    const int head_in = a.lane_head[tid];
    const int row0_in = a.lane_row0[tid];

#ifdef QL_PHASE_STAMPS
    uint64_t st_acc[NUM_STAMPS];
    for (int i = 0; i < NUM_STAMPS; ++i) st_acc[i] = 0;
    uint64_t st_last = __builtin_amdgcn_s_memtime();
#endif
    for (;;) {
        if (tid == 0) *s_frame = claim_frame(a);
        STAMP(ST_SETUP);
        __syncthreads();
        STAMP(ST_SETUP_WAIT);
        const int f = __builtin_amdgcn_readfirstlane(*s_frame);  // wave-uniform: SGPR addressing
        if (f >= a.batch) break;
        uint64_t clk0 = 0;  // the trial's own span inside the batch (a.frame_clk)
        if (tid == 0 && a.frame_clk) clk0 = __builtin_amdgcn_s_memrealtime();
        const double *llr = a.llr + (size_t)f * n;
        const uint8_t *sy = a.synd + (size_t)f * m;
        for (int j = tid; j < m; j += T) rowflag[j] = sy[j] & 1;
        if constexpr (ADAPT)
            for (int i = tid; i < n; i += T) total[i] = 0.0;  // total_bit_llr starts zeroed
        __syncthreads();

        int iters = a.max_it, okv = 0;
        bool had_vn = false;
        for (int it = 0;; ++it) {
            // ---- syndrome check of the current decision --------------------------
            // SPA/SPA-lin/NMSA/OMSA: after each VN (:86,101-107), so at the top of
            // it >= 1 and once more after the last iteration.  ANMSA/AOMSA: inside
            // the CN pass of every iteration, on the previous decisions (:745-776).
            const bool needS = ADAPT ? (it < a.max_it) : (it > 0);
            if (needS) {
                int mis = 0;
                for (int j = tid; j < m; j += T) {
                    const int deg = a.row_deg[j];
                    int par = 0;
                    for (int k = 0; k < deg; ++k) {
                        const int c = a.ell_col[(size_t)k * m + j];
                        const double z = had_vn ? total[c] : llr[c];
                        par ^= (z <= 0.0) ? 1 : 0;
                    }
                    const uint8_t fl = rowflag[j];
                    const int rm = (par ^ fl) & 1;
                    rowflag[j] = (uint8_t)((fl & 5) | (rm << 1));
                    mis |= rm;
                }
                STAMP(ST_S);
                const int anymis = __syncthreads_or(mis);
                STAMP(ST_S_WAIT);
                if (!anymis) {
                    iters = ADAPT ? it + 1 : it;
                    okv = 1;
                    break;
                }
            }
            if (it == a.max_it) break;

            // Re-opaque the lane constants each iteration: per-slot masks derived
            // from them (k < head, ...) are then computed at their use instead
            // of being hoisted out of the frame loop into ~80 SGPRs.
            int head = head_in, row0 = row0_in;
            asm volatile("" : "+v"(head), "+v"(row0));

            // ---- CN phase 1: b2c, tanh / row aggregates over this lane's edges ----
            int r = row0;
            double acc = 0.0;
            MinAgg ag, hag;
            agg_init(ag);
            agg_init(hag);
            bool tail_open = false;
            meta.each(EPL, [&](int k, uint32_t mt) {
                if (!(mt & META_VALID)) return;
                if (k > 0 && (mt & META_START)) ++r;
                const int col = (int)(mt & META_COL_MASK);
                double x;
                if (it == 0) {
                    x = llr[col];  // initial b2c = channel LLR, unclipped (:21-29)
                } else {
                    // VN extrinsic (:115); occurrence pairing: computed by the
                    // pairing pass below from the edge the counters pair it with
                    if (pbuf) x = pbuf[(size_t)k * T + tid];
                    else x = total[col] - c2b.get(k);
                    if (thr_on) x = clip_msg(x, thr);
                }
                if constexpr (SPA_FAM) {
                    const double t = (ALG == 0) ? ql_exact::tanh_dec(x / 2.) : tanh_lin(x / 2.);
                    c2b.set(k, t);
                    if (k < head) return;
                    if (mt & META_START) acc = ((rowflag[r] & 1) ? -1. : 1.) * t;  // :57-62
                    else acc = acc * t;
                    if (mt & META_END) rowA[r] = acc;
                    tail_open = !(mt & META_END);
                } else {
                    c2b.set(k, x);
                    if (k < head) {
                        agg_push(hag, x);
                        return;
                    }
                    if (mt & META_START) agg_init(ag);
                    agg_push(ag, x);
                    if (mt & META_END) {
                        rowA[r] = ag.m1;
                        rowB[r] = ag.m2;
                        rowflag[r] = (uint8_t)((rowflag[r] & 3) | (ag.neg << 2));
                    }
                    tail_open = !(mt & META_END);
                }
            });
            if (tail_open) {
                if constexpr (SPA_FAM) {
                    carryA[tid] = acc;
                } else {
                    carryA[tid] = ag.m1;
                    carryB[tid] = ag.m2;
                    carryI[tid] = ag.neg;
                }
            }
            STAMP(ST_CN1);
            __syncthreads();
            STAMP(ST_CN1_WAIT);

            // ---- CN phase 2: finish rows begun in the previous lane ----------------
            if (head > 0) {
                if constexpr (SPA_FAM) {
                    double p = carryA[tid - 1];
                    if constexpr (R > 0) {
#pragma unroll
                        for (int k = 0; k < R; ++k)
                            if (k < head) p = p * c2b.get(k);
                    } else {
                        for (int k = 0; k < head; ++k) p = p * c2b.get(k);
                    }
                    rowA[row0] = p;
                } else {
                    MinAgg t;
                    t.m1 = carryA[tid - 1];
                    t.m2 = carryB[tid - 1];
                    t.neg = carryI[tid - 1];
                    agg_merge(t, hag);
                    rowA[row0] = t.m1;
                    rowB[row0] = t.m2;
                    rowflag[row0] = (uint8_t)((rowflag[row0] & 3) | (t.neg << 2));
                }
            }
            STAMP(ST_CN2);
            __syncthreads();
            STAMP(ST_CN2_WAIT);

            // ---- CN phase 3: check-to-bit messages, clipped (:64-74 etc.) ---------
            r = row0;
            meta.each(EPL, [&](int k, uint32_t mt) {
                if (!(mt & META_VALID)) return;
                if (k > 0 && (mt & META_START)) ++r;
                double c;
                if constexpr (SPA_FAM) {
                    const double prod = rowA[r] / c2b.get(k);  // :66
                    c = 2. * ((ALG == 0) ? ql_exact::atanh_dec(prod) : atanh_lin(prod));
                } else {
                    const double x = c2b.get(k);
                    const uint8_t fl = rowflag[r];
                    double sp = (fl & 1) ? -1. : 1.;  // :376
                    sp *= ((fl >> 2) & 1) ? -1. : 1.;  // :398
                    const double prod = sp * ((x > 0) ? 1. : -1.);  // :402
                    const double m1 = rowA[r];
                    const double sel = (fabs(x) == m1) ? rowB[r] : m1;  // :406
                    double fac = a.primary;
                    if (ADAPT && (fl & 2)) fac = a.secondary;  // :749-757
                    if constexpr (NORM) {
                        c = fac * prod * sel;  // :405-406
                    } else {
                        const double d = sel - fac;  // :573-574
                        c = prod * ((d < 0.) ? 0. : d);
                    }
                }
                if (thr_on) c = clip_msg(c, thr);
                c2b.set(k, c);
            });

            STAMP(ST_CN3);
            // ---- VN: totals in std::accumulate order (:76-84) -----------------------
            for (int i = tid; i < n; i += T) total[i] = llr[i];
            STAMP(ST_VN0);
            __syncthreads();
            STAMP(ST_VN0_WAIT);
            for (int kk = 0; kk < a.dv_max; ++kk) {
                meta.each(EPL, [&](int k, uint32_t mt) {
                    if ((mt & META_VALID) && ((mt >> META_KPOS_SHIFT) & META_KPOS_MASK) == (uint32_t)kk) {
                        const int col = (int)(mt & META_COL_MASK);
                        total[col] = total[col] + c2b.get(k);
                    }
                });
                STAMP(ST_VNK);
                __syncthreads();
                STAMP(ST_VNK_WAIT);
            }
            if constexpr (R == 0) {
                // Occurrence pairing (:109-120 with unsorted lists): input slot s
                // of the next check-node pass takes total[i] - c2b of the edge
                // the reference's counters pair it with (another lane's slot).
                // The messages stay untouched until the next scan, after the barrier.
                if (pbuf) {
                    meta.each(EPL, [&](int k, uint32_t mt) {
                        if (!(mt & META_VALID)) return;
                        const size_t s = (size_t)k * T + tid;
                        pbuf[s] = total[a.pair_col[s]] - wg[a.pair_src[s]];
                    });
                    __syncthreads();
                }
            }
            had_vn = true;
        }

        // ---- outputs: bit_array_out, decoding_result, total_bit_llr ----------------
        uint8_t *bits = a.bits + (size_t)f * n;
        double *post = a.post ? a.post + (size_t)f * n : nullptr;
        for (int i = tid; i < n; i += T) {
            const double z = had_vn ? total[i] : llr[i];
            bits[i] = (z <= 0.0) ? 1 : 0;
            if (post) post[i] = total[i];
        }
        if (tid == 0) {
            a.iters[f] = (uint32_t)iters;
            a.ok[f] = (uint8_t)okv;
            if (a.frame_clk) {
                a.frame_clk[2 * (size_t)f] = clk0;
                a.frame_clk[2 * (size_t)f + 1] = __builtin_amdgcn_s_memrealtime();
            }
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

// ---- QKD_LDPC frame construction (src/qkd_ldpc_algorithm.cpp:1043-1052) --------
// One workgroup per frame.  Alice's and Bob's keys are first packed into LDS
// bit words (dev::pack_key_bits: coalesced 16-byte loads), so the palette
// codes' gather by label (col_orig) and the syndrome's row gathers read LDS.
__global__ void __launch_bounds__(1024) build_frames_kernel(int n, int m, const int32_t *ell_col,
                                                           const int32_t *row_deg, const uint8_t *alice,
                                                           const uint8_t *bob, const double *log_p,
                                                           double *llr, uint8_t *synd, uint8_t *codes,
                                                           double *palette, uint8_t *pal_ok,
                                                           const int32_t *col_orig) {
    extern __shared__ uint32_t kb[];
    const int nw = (n + 31) / 32;
    uint32_t *abits = kb, *bbits = kb + nw;
    const size_t f = blockIdx.x;
    const double lp = log_p[f];
    const uint8_t *al = alice + f * (size_t)n;
    const uint8_t *bo = bob + f * (size_t)n;
    dev::pack_key_bits(al, n, abits);
    dev::pack_key_bits(bo, n, bbits);
    __syncthreads();
    if (llr) {
        double *l = llr + f * (size_t)n;
        for (int i = threadIdx.x; i < n; i += blockDim.x) l[i] = dev::key_bit(bbits, i) ? -lp : lp;
    }
    if (codes) {  // V2 palette form: code 0 = +log_p, 1 = -log_p; in label order (col_orig)
        const int nc = (n + 3) / 4;
        uint8_t *cs = codes + f * (size_t)nc;
        for (int j = threadIdx.x; j < nc; j += blockDim.x) {
            int byte = 0;
            for (int s = 0; s < 4; ++s) {
                const int i = 4 * j + s;
                if (i < n && dev::key_bit(bbits, col_orig ? col_orig[i] : i)) byte |= 1 << (2 * s);
            }
            cs[j] = (uint8_t)byte;
        }
        if (threadIdx.x < 4) palette[f * 4 + threadIdx.x] = threadIdx.x == 1 ? -lp : lp;  // unused 2, 3 repeat entry 0
        if (threadIdx.x == 0) pal_ok[f] = 1;
    }
    uint8_t *s = synd + f * (size_t)m;
    for (int j = threadIdx.x; j < m; j += blockDim.x) s[j] = (uint8_t)dev::row_parity(abits, ell_col, row_deg, m, j);
}

// keys_match = arrays_equal(alice, bob_solution) (src/qkd_ldpc_algorithm.cpp:1087):
// 16 bytes per load where both rows are 16-byte aligned (n % 16 == 0).
__global__ void __launch_bounds__(1024) keys_match_kernel(int n, const uint8_t *alice, const uint8_t *bits,
                                                          uint8_t *match) {
    const size_t f = blockIdx.x;
    const uint8_t *a = alice + f * (size_t)n, *b = bits + f * (size_t)n;
    int diff = 0;
    if (n % 16 == 0 && ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) == 0) {
        const uint4 *a4 = reinterpret_cast<const uint4 *>(a), *b4 = reinterpret_cast<const uint4 *>(b);
        for (int i = threadIdx.x; i < n / 16; i += blockDim.x) {
            const uint4 x = a4[i], y = b4[i];
            diff |= ((x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w)) != 0;
        }
    } else {
        for (int i = threadIdx.x; i < n; i += blockDim.x) diff |= (a[i] != b[i]);
    }
    diff = __syncthreads_or(diff);
    if (threadIdx.x == 0) match[f] = diff ? 0 : 1;
}

__global__ void __launch_bounds__(256) math_selftest_kernel(int fn, int count, const double *in, double *out) {
    __shared__ ql_exact::Expm1A ctab_a[ql_exact::EXPM1_CLASSES];  // fn 8: the SPA scan's table form
    __shared__ ql_exact::Expm1B ctab_b[ql_exact::EXPM1_CLASSES];
    if (threadIdx.x < ql_exact::EXPM1_CLASSES)
        ql_exact::expm1_class(threadIdx.x + ql_exact::EXPM1_K_MIN, &ctab_a[threadIdx.x], &ctab_b[threadIdx.x]);
    const ql_exact::Expm1Tab ctab{ctab_a, ctab_b, 1};
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const double x = in[i];
    double y;
    int flag = 0;
    switch (fn) {
    case 8: y = ql_exact::tanh_half_clip_t(x, 44.0, 1.0, &flag, ctab); break;  // tanh(clip(x, inf) / 2.), tanh(22) = 1
    case 9:  // the SPA message pass's clip(2. * atanh(x), 100)
        y = ql_exact::atanh2_clip(x, 100.0, ql_exact::atanh2_full(0x1.fffffffffffffp-1));
        break;
    case 0: y = ql_exact::tanh_exact(x); break;
    case 1: y = ql_exact::atanh_exact(x); break;
    case 2: y = ql_exact::expm1_exact(x); break;
    case 3: y = ql_exact::log1p_exact(x); break;
    case 4: y = tanh_lin(x); break;
    case 5: y = atanh_lin(x); break;
    case 6: y = ql_exact::tanh_dec(x); break;
    default: y = ql_exact::atanh_dec(x); break;
    }
    out[i] = y;
}

using KernelFn = void (*)(DecodeArgs);

template <int ALG>
KernelFn pick(int variant) {
    switch (variant) {
    case VAR_REG_LDS: return decode_kernel<ALG, EPL_REG, true>;
    case VAR_GLB_LDS: return decode_kernel<ALG, 0, true>;
    default: return decode_kernel<ALG, 0, false>;
    }
}

KernelFn kernel_for(int variant, int alg) {
    switch (alg) {
    case 0: return pick<0>(variant);
    case 1: return pick<1>(variant);
    case 2: return pick<2>(variant);
    case 3: return pick<3>(variant);
    case 4: return pick<4>(variant);
    default: return pick<5>(variant);
    }
}

}  // namespace

size_t lds_bytes_for(int variant, int n, int m, int T) {
    if (variant == VAR_GLB_GLB) return CTRL_BYTES;
    return CTRL_BYTES + FrameLayout(n, m, T).bytes;
}

long long scratch_doubles_for(int variant, int n, int m, int T, int EPL) {
    long long d = 0;
    if (variant != VAR_REG_LDS) d += (long long)EPL * T;
    if (variant == VAR_GLB_GLB) d += (long long)((FrameLayout(n, m, T).bytes + 7) / 8);
    return d;
}

hipError_t allow_dynamic_lds(const void *k, size_t bytes) {
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, size_t> limit;  // the largest value set per (device, kernel)
    int dev = 0;
    const hipError_t de = hipGetDevice(&dev);
    if (de != hipSuccess) return de;
    std::lock_guard<std::mutex> lk(mu);
    size_t &cur = limit[{dev, k}];
    if (bytes <= cur) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) cur = bytes;
    return e;
}

hipError_t launch_decode(int variant, const DecodeArgs &a, int workgroups, size_t lds_bytes,
                         hipStream_t stream) {
    KernelFn k = kernel_for(variant, a.alg);
    hipError_t e = allow_dynamic_lds(reinterpret_cast<const void *>(k), lds_bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(workgroups), dim3(a.T), lds_bytes, stream, a);
    return hipGetLastError();
}

hipError_t occupancy(int variant, int alg, int T, size_t lds_bytes, int *blocks_per_cu) {
    KernelFn k = kernel_for(variant, alg);
    hipError_t e = allow_dynamic_lds(reinterpret_cast<const void *>(k), lds_bytes);
    if (e != hipSuccess) return e;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k, T, lds_bytes);
}

hipError_t launch_build_frames(int n, int m, int max_dc, const int32_t *ell_col, const int32_t *row_deg,
                               int batch, const uint8_t *alice, const uint8_t *bob, const double *log_p,
                               double *llr, uint8_t *synd, uint8_t *codes, double *palette, uint8_t *pal_ok,
                               const int32_t *col_orig, hipStream_t stream) {
    (void)max_dc;
    if (batch <= 0) return hipSuccess;
    const size_t lds = build_frames_lds(n);  // the two keys as bit words
    if (lds > LDS_MAX_BYTES) return hipErrorInvalidValue;
    if (lds > 65536) {
        hipError_t e = allow_dynamic_lds(reinterpret_cast<const void *>(build_frames_kernel), lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(build_frames_kernel, dim3(batch), dim3(aux_frame_threads(n)), lds, stream, n, m, ell_col, row_deg, alice,
                       bob, log_p, llr, synd, codes, palette, pal_ok, col_orig);
    return hipGetLastError();
}

hipError_t launch_math_selftest(int fn, int count, const double *in, double *out, hipStream_t stream) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(math_selftest_kernel, dim3((count + 255) / 256), dim3(256), 0, stream, fn, count, in, out);
    return hipGetLastError();
}

hipError_t launch_keys_match(int batch, int n, const uint8_t *alice, const uint8_t *bits, uint8_t *match,
                             hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    hipLaunchKernelGGL(keys_match_kernel, dim3(batch), dim3(aux_frame_threads(n)), 0, stream, n, alice, bits, match);
    return hipGetLastError();
}

}  // namespace qldpc
