// decoder_common.hpp — device helpers shared by the decoder kernels.
#pragma once
#include <float.h>

#include "decoder.hpp"
#include "exact_math.h"

// Diagnostic build only (-DQL_PHASE_STAMPS): per-wave s_memtime accumulators
// of every phase's work and barrier-wait time, written to DecodeArgs::stamps.
#ifdef QL_PHASE_STAMPS
#define STAMP(id)                                                \
    do {                                                         \
        const uint64_t _t = __builtin_amdgcn_s_memtime();        \
        st_acc[id] += _t - st_last;                              \
        st_last = _t;                                            \
    } while (0)
#else
#define STAMP(id) ((void)0)
#endif

namespace qldpc {
namespace dev {

// A frame's key bytes (0 / 1 each) packed into LDS bit words by the whole
// workgroup: word w holds bits 32 w .. 32 w + 31.  With n % 32 == 0 and a
// 16-byte aligned key, each word is two 16-byte loads (a wave reads 2 KiB
// contiguously); otherwise byte loads.  The frame builders then gather key
// bits from LDS instead of bytes from L2.
__device__ __forceinline__ uint32_t pack4(uint32_t x) {  // 4 bytes of 0 / 1 -> 4 bits
    return (x & 1u) | ((x >> 7) & 2u) | ((x >> 14) & 4u) | ((x >> 21) & 8u);
}
__device__ inline void pack_key_bits(const uint8_t *key, int n, uint32_t *bits) {
    const int nw = (n + 31) / 32;
    const bool wide = (n % 32 == 0) && ((reinterpret_cast<uintptr_t>(key) & 15) == 0);
    for (int w = threadIdx.x; w < nw; w += blockDim.x) {
        uint32_t v = 0;
        if (wide) {
            const uint4 *k4 = reinterpret_cast<const uint4 *>(key) + 2 * w;
            const uint4 lo = k4[0], hi = k4[1];
            v = pack4(lo.x) | (pack4(lo.y) << 4) | (pack4(lo.z) << 8) | (pack4(lo.w) << 12) | (pack4(hi.x) << 16) |
                (pack4(hi.y) << 20) | (pack4(hi.z) << 24) | (pack4(hi.w) << 28);
        } else {
            for (int b = 0; b < 32 && 32 * w + b < n; ++b) v |= (uint32_t)(key[32 * w + b] & 1u) << b;
        }
        bits[w] = v;
    }
}
__device__ __forceinline__ uint32_t key_bit(const uint32_t *bits, int i) { return (bits[i >> 5] >> (i & 31)) & 1u; }
// calculate_syndrome's row j (src/array_and_matrix_operations.cpp:936-950)
// over a frame's bits in LDS (row-ELL columns, [k][m]): the column loads are
// issued four at a time (independent L2 loads in flight, not one per XOR).
__device__ __forceinline__ uint32_t row_parity(const uint32_t *bits, const int32_t *ell_col, const int32_t *row_deg,
                                               int m, int j) {
    uint32_t p = 0;
    const int deg = row_deg[j];
    int k = 0;
    for (; k + 4 <= deg; k += 4) {
        int c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) c[q] = ell_col[(size_t)(k + q) * m + j];
#pragma unroll
        for (int q = 0; q < 4; ++q) p ^= key_bit(bits, c[q]);
    }
    for (; k < deg; ++k) p ^= key_bit(bits, ell_col[(size_t)k * m + j]);
    return p;
}

// threshold_matrix (src/array_and_matrix_operations.cpp:953-972): v > thr -> thr,
// v < -thr -> -thr, NaN passes.  With thr > 0 that is |v| > thr -> copysign(thr, v):
// one compare (abs modifier), one bfi and two selects.
__device__ __forceinline__ double clip_msg(double v, double thr) {
    return (__builtin_fabs(v) > thr) ? __builtin_copysign(thr, v) : v;
}

// tanh_lin_approx / atanh_lin_approx (src/qkd_ldpc_algorithm.cpp:146-172).
__device__ __forceinline__ double tanh_lin(double x) {
    const double a = fabs(x);
    double r;
    if (a < 0.5) r = 0.9242 * a;
    else if (a < 0.9) r = 0.6355 * a + 0.1444;
    else if (a < 1.2) r = 0.3912 * a + 0.3642;
    else if (a < 1.75) r = 0.1958 * a + 0.5986;
    else if (a < 2.5) r = 0.0603 * a + 0.8358;
    else if (a < 3.5) r = 0.0115 * a + 0.9577;
    else if (a < 8) r = 0.0004 * a + 0.9967;
    else r = 1;
    return (x < 0.) ? -r : r;
}
__device__ __forceinline__ double atanh_lin(double x) {
    const double a = fabs(x);
    double r;
    if (a < 0.7) r = 1.196 * a - 0.0323;
    else if (a < 0.9) r = 2.9187 * a - 1.214;
    else if (a < 0.999) r = 10.8717 * a - 8.3717;
    else r = 2510.9 * a - 2505.9;
    return (x < 0.) ? -r : r;
}

// Min-sum row aggregate: parity of x<0, and the two smallest |x| with the
// reference's strict-< scan (src/qkd_ldpc_algorithm.cpp:381-397).  The scan's
// result is the two smallest of {|x| : |x| < DBL_MAX} padded with DBL_MAX, so
// partial aggregates merge order-free (exact).
struct MinAgg {
    double m1, m2;
    int neg;
};
__device__ __forceinline__ void agg_init(MinAgg &a) {
    a.m1 = DBL_MAX;
    a.m2 = DBL_MAX;
    a.neg = 0;
}
__device__ __forceinline__ void agg_push(MinAgg &a, double x) {
    if (x < 0) a.neg ^= 1;
    const double ax = fabs(x);
    if (ax < a.m1) {
        a.m2 = a.m1;
        a.m1 = ax;
    } else if (ax < a.m2) {
        a.m2 = ax;
    }
}
__device__ __forceinline__ void agg_merge(MinAgg &a, const MinAgg &b) {
    a.neg ^= b.neg;
    const bool bl = b.m1 < a.m1;
    const double lo = bl ? b.m1 : a.m1;
    const double hi = bl ? a.m1 : b.m1;
    const double m2 = (a.m2 < b.m2) ? a.m2 : b.m2;
    a.m1 = lo;
    a.m2 = (hi < m2) ? hi : m2;
}

// Per-edge message storage of one lane.
template <int R>
struct EdgeMsgs {  // VGPR-resident: R slots, indexed only by unrolled constants
    double v[R];
    __device__ __forceinline__ void bind(double *, int, int) {}
    __device__ __forceinline__ double get(int k) const { return v[k]; }
    __device__ __forceinline__ void set(int k, double x) { v[k] = x; }
};
template <>
struct EdgeMsgs<0> {  // per-workgroup global scratch, slot-major [k][lane]: coalesced
    double *p;
    int T;
    __device__ __forceinline__ void bind(double *base, int tid, int TT) {
        p = base + tid;
        T = TT;
    }
    __device__ __forceinline__ double get(int k) const { return p[(size_t)k * T]; }
    __device__ __forceinline__ void set(int k, double x) { p[(size_t)k * T] = x; }
};

// V2 message storage: slots k < R - RL in VGPRs, slots R - RL <= k < R in
// LDS, slot-major [k - (R - RL)][lane] (lane stride LS, the workgroup's lanes:
// conflict-free 8-byte rows, constant offsets from one base register), and slots
// R <= k < R + RG in this workgroup's global scratch, slot-major [k - R][lane]
// — coalesced, constant offsets, L2/MALL-resident.  A lane only ever reads
// back what it wrote itself, so program order suffices.  The LDS slots keep
// the register kernel within 128 VGPRs without compiler spills (scratch
// stores whose reloads wait on the vector-memory counter).
template <int R, int RG, int RL = 0, int LS = REG_TSTRIDE>
struct EdgeMsgsH {
    static constexpr int RV = R - RL;
    double v[RV];
    __amdgpu_buffer_rsrc_t rs;
    int voff;
    double *lp;
    __device__ __forceinline__ void bind(double *wg_base, int tid) {
        if constexpr (RG > 0) {
            rs = __builtin_amdgcn_make_buffer_rsrc((void *)wg_base, (short)0, RG * REG_TSTRIDE * 8, 0x00020000);
            voff = tid * 8;
        }
    }
    __device__ __forceinline__ void bind_lds(double *lds_base, int tid) {
        if constexpr (RL > 0) lp = lds_base + tid;
    }
    __device__ __forceinline__ double get(int k) const {
        if (k < RV) return v[k];
        if (k < R) return lp[(k - RV) * LS];
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, (k - R) * REG_TSTRIDE * 8, 0));
    }
    // For passes that visit every slot in order (the check-node scan, the
    // message pass): the scratch slots of a group of four are requested
    // together at the group's first slot, so their four L2 round trips overlap
    // instead of each load waiting out the previous slot's store.
    // (one group ahead instead, 8 more VGPRs: C5 +10%, spills)
    double pre[4];
    __device__ __forceinline__ double get_seq(int k) {
        if constexpr (RG > 0) {
            static_assert(R % 4 == 0 && RG % 4 == 0, "scratch slots come in groups of four");
            if (k >= R) {
                const int j = k - R;
                if ((j & 3) == 0) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) pre[q] = get(k + q);
                }
                return pre[j & 3];
            }
        }
        return get(k);
    }
    __device__ __forceinline__ void set(int k, double x) {
        if (k < RV) {
            v[k] = x;
        } else if (k < R) {
            lp[(k - RV) * LS] = x;
        } else {
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, x), rs, voff, (k - R) * REG_TSTRIDE * 8,
                                                  0);
        }
    }
};

// Visit this lane's slots in order, handing each slot's metadata word to f.
// Metadata is one uint4 per four consecutive slots, group-major [g][lane], so a
// wave reads 1 KiB contiguous per group.  The register variant uses a fixed
// group stride of REG_TSTRIDE lanes and buffer loads whose group offset is a
// compile-time constant: no per-group address stays live across the kernel.
#ifdef QL_SLOT_FENCE
#define QL_SLOT_BARRIER() __builtin_amdgcn_sched_barrier(0)
#else
#define QL_SLOT_BARRIER() ((void)0)
#endif

template <int R>
struct MetaSrc {
    __amdgpu_buffer_rsrc_t rs;
    int voff;
    __device__ __forceinline__ void init(const uint32_t *base, int tid, int) {
        rs = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (R / 4) * REG_TSTRIDE * 16, 0x00020000);
        voff = tid * 16;
    }
    template <typename F>
    __device__ __forceinline__ void each(int, F &&f) const {
        static_assert(R % 4 == 0, "register slots come in groups of four");
#pragma unroll
        for (int g = 0; g < R / 4; ++g) {
            const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, g * REG_TSTRIDE * 16, 0);
            f(4 * g + 0, (uint32_t)q[0]);
            QL_SLOT_BARRIER();
            f(4 * g + 1, (uint32_t)q[1]);
            QL_SLOT_BARRIER();
            f(4 * g + 2, (uint32_t)q[2]);
            QL_SLOT_BARRIER();
            f(4 * g + 3, (uint32_t)q[3]);
            QL_SLOT_BARRIER();
        }
    }
};
// a + b + (this lane's bit of the lane mask m): one v_addc with the mask as
// carry-in (the compiler otherwise materialises the bit: a select and an add).
__device__ __forceinline__ uint32_t add_carry(uint32_t a, uint32_t b, uint64_t m) {
    uint32_t r;
    uint64_t co;
    asm("v_addc_co_u32_e64 %0, %1, %2, %3, %4" : "=v"(r), "=s"(co) : "v"(a), "v"(b), "s"(m));
    (void)co;
    return r;
}
__device__ __forceinline__ int add_carry(int a, int b, uint64_t m) {
    return (int)add_carry((uint32_t)a, (uint32_t)b, m);
}

// Read-only for a kernel's lifetime: loads through this type are scalar (s_load).
typedef const __attribute__((address_space(4))) uint64_t cu64_t;

// Issue priority of a SIMD's waves, rotated slot group by slot group: the
// sequencer otherwise favours the oldest wave, so a SIMD's four waves finish a
// phase one after another and the last runs alone (one wave cannot issue
// dependent FP64 back to back).  Rotating the favoured wave keeps them level.
// A SIMD holds waves w, w + 4, w + 8, w + 12 of a workgroup, told apart by
// w >> 2; the rotation runs backwards through them (measured: C2 SPA -5.6%,
// C3 OMSA -3%, same-box A/B; also in the message pass and the VN phases:
// C3 a further -1.6%, C5 R=0.5 -0.8%).
__device__ __forceinline__ void rotate_prio(int g) {
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 8));
    switch ((3 * g + wv) & 3) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
    }
}

// Same, but only the slots a wave actually holds: `epl_s` is wave-uniform (an
// SGPR), so each slot costs a scalar compare-and-branch, no VALU.  Slots past
// a lane's last row are dummies, but a lane whose last row continues into the
// next lane must never see one (it would enter that row's running product).
template <int R>
struct MetaSrcW : MetaSrc<R> {
    template <typename F>
    __device__ __forceinline__ void each_upto(int epl_s, F &&f) const {
        // opaque per call: keeps the slot guards scalar compares instead of
        // 40 hoisted lane masks (which spill into VGPR lanes: 2 VALU per slot)
        asm volatile("" : "+s"(epl_s));
#pragma unroll
        for (int g = 0; g < R / 4; ++g) {
            rotate_prio(g);
            if (4 * g < epl_s) {
                const auto q = __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff, g * REG_TSTRIDE * 16, 0);
                f(4 * g + 0, (uint32_t)q[0]);
                if (4 * g + 1 < epl_s) f(4 * g + 1, (uint32_t)q[1]);
                if (4 * g + 2 < epl_s) f(4 * g + 2, (uint32_t)q[2]);
                if (4 * g + 3 < epl_s) f(4 * g + 3, (uint32_t)q[3]);
            }
        }
    }
    // Same, with a per-slot value ld(mt) (a total in global memory) loaded for
    // the group's four slots before any of them is visited, and the next
    // group's metadata requested before this group's work: one memory latency
    // per group instead of two per slot.
    template <typename LD, typename F>
    __device__ __forceinline__ void each_upto_tv(int epl_s, LD &&ld, F &&f) const {
        asm volatile("" : "+s"(epl_s));
        auto q = __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff, 0, 0);
#pragma unroll
        for (int g = 0; g < R / 4; ++g) {
            rotate_prio(g);
            if (4 * g < epl_s) {
                double tv[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) tv[i] = ld((uint32_t)q[i]);  // slots past epl: dummy column
                const auto qn = (g + 1 < R / 4)
                                    ? __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff,
                                                                            (g + 1) * REG_TSTRIDE * 16, 0)
                                    : q;
                f(4 * g + 0, (uint32_t)q[0], tv[0]);
                if (4 * g + 1 < epl_s) f(4 * g + 1, (uint32_t)q[1], tv[1]);
                if (4 * g + 2 < epl_s) f(4 * g + 2, (uint32_t)q[2], tv[2]);
                if (4 * g + 3 < epl_s) f(4 * g + 3, (uint32_t)q[3], tv[3]);
                q = qn;
            }
        }
    }
    // Same as each_upto, also handing over the word of a second metadata array
    // of identical layout (rs2).
    template <typename F>
    __device__ __forceinline__ void each_upto2(int epl_s, __amdgpu_buffer_rsrc_t rs2, F &&f) const {
        asm volatile("" : "+s"(epl_s));
#pragma unroll
        for (int g = 0; g < R / 4; ++g) {
            rotate_prio(g);
            if (4 * g < epl_s) {
                const auto q = __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff, g * REG_TSTRIDE * 16, 0);
                const auto q2 = __builtin_amdgcn_raw_buffer_load_b128(rs2, this->voff, g * REG_TSTRIDE * 16, 0);
                f(4 * g + 0, (uint32_t)q[0], (uint32_t)q2[0]);
                if (4 * g + 1 < epl_s) f(4 * g + 1, (uint32_t)q[1], (uint32_t)q2[1]);
                if (4 * g + 2 < epl_s) f(4 * g + 2, (uint32_t)q[2], (uint32_t)q2[2]);
                if (4 * g + 3 < epl_s) f(4 * g + 3, (uint32_t)q[3], (uint32_t)q2[3]);
            }
        }
    }
    // Same, with the next group's two metadata words requested before this
    // group's work.  For passes that store to global memory per slot (the VN
    // stage of split frames and the hybrid shape): on gfx9 vmcnt counts stores
    // too and drains in issue order, so a metadata load issued after a group's
    // stores cannot be waited for without waiting for those stores; requested
    // one group early, it waits only for the stores of the group before.
    template <typename F>
    __device__ __forceinline__ void each_upto2_pf(int epl_s, __amdgpu_buffer_rsrc_t rs2, F &&f) const {
        asm volatile("" : "+s"(epl_s));
        auto q = __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff, 0, 0);
        auto q2 = __builtin_amdgcn_raw_buffer_load_b128(rs2, this->voff, 0, 0);
#pragma unroll
        for (int g = 0; g < R / 4; ++g) {
            rotate_prio(g);
            if (4 * g < epl_s) {
                const bool more = g + 1 < R / 4 && 4 * (g + 1) < epl_s;
                const auto qn = more ? __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff,
                                                                             (g + 1) * REG_TSTRIDE * 16, 0)
                                     : q;
                const auto q2n = more ? __builtin_amdgcn_raw_buffer_load_b128(rs2, this->voff,
                                                                              (g + 1) * REG_TSTRIDE * 16, 0)
                                      : q2;
                f(4 * g + 0, (uint32_t)q[0], (uint32_t)q2[0]);
                if (4 * g + 1 < epl_s) f(4 * g + 1, (uint32_t)q[1], (uint32_t)q2[1]);
                if (4 * g + 2 < epl_s) f(4 * g + 2, (uint32_t)q[2], (uint32_t)q2[2]);
                if (4 * g + 3 < epl_s) f(4 * g + 3, (uint32_t)q[3], (uint32_t)q2[3]);
                q = qn;
                q2 = q2n;
            }
        }
    }
    // Groups of four slots at least one of which is in the mask: f(g, q, bits)
    // with q the group's four metadata words and bits its 4-bit slice of the mask.
    template <typename F>
    __device__ __forceinline__ void each_group_masked(uint32_t mlo, uint32_t mhi, F &&f) const {
#pragma unroll
        for (int g = 0; g < R / 4; ++g) {
            rotate_prio(g);
            const uint32_t w = (4 * g < 32) ? mlo : mhi;
            const uint32_t bits = (w >> ((4 * g) & 31)) & 15u;
            if (bits) {
                const auto q = __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff, g * REG_TSTRIDE * 16, 0);
                f(g, q, bits);
            }
        }
    }
    // Same, with the next group's metadata requested before this group's work
    // (a VN phase does little per group: one memory latency per group would
    // otherwise be exposed on every wave at once).
    template <typename F>
    __device__ __forceinline__ void each_group_masked_pf(uint32_t mlo, uint32_t mhi, F &&f) const {
        auto q = __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff, 0, 0);
#pragma unroll
        for (int g = 0; g < R / 4; ++g) {
            const uint32_t w = (4 * g < 32) ? mlo : mhi;
            const uint32_t bits = (w >> ((4 * g) & 31)) & 15u;
            const auto qn = (g + 1 < R / 4)
                                ? __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff, (g + 1) * REG_TSTRIDE * 16, 0)
                                : q;
            if (bits) f(g, q, bits);
            q = qn;
        }
    }
    // Batches of NB consecutive groups at least one of which is in the mask:
    // f(g, q[NB], nv) — q[j] the metadata of group g + j, nv the groups that
    // exist.  The next batch's first group's metadata is requested before
    // this batch's work.
    template <int NB, typename F>
    __device__ __forceinline__ void each_group_batch_masked_pf(uint32_t mlo, uint32_t mhi, F &&f) const {
        constexpr int NG = R / 4;
        auto q0 = __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff, 0, 0);
#pragma unroll
        for (int g = 0; g < NG; g += NB) {
            uint32_t bits = 0;
            decltype(q0) q[NB];
            q[0] = q0;
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                if (g + j < NG) {
                    const uint32_t w = (4 * (g + j) < 32) ? mlo : mhi;
                    bits |= (w >> ((4 * (g + j)) & 31)) & 15u;
                    if (j > 0)
                        q[j] = __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff, (g + j) * REG_TSTRIDE * 16, 0);
                } else {
                    q[j] = q0;
                }
            }
            const auto qn = (g + NB < NG)
                                ? __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff, (g + NB) * REG_TSTRIDE * 16, 0)
                                : q0;
            if (bits) f(g, q, (NG - g < NB) ? NG - g : NB);
            q0 = qn;
        }
    }
    template <typename F>
    __device__ __forceinline__ void each_masked(uint32_t mlo, uint32_t mhi, F &&f) const {
#pragma unroll
        for (int g = 0; g < R / 4; ++g) {
            const uint32_t w = (4 * g < 32) ? mlo : mhi;
            const int b = (4 * g) & 31;
            if ((w >> b) & 15u) {
                const auto q = __builtin_amdgcn_raw_buffer_load_b128(this->rs, this->voff, g * REG_TSTRIDE * 16, 0);
                if ((w >> b) & 1u) f(4 * g + 0, (uint32_t)q[0]);
                if ((w >> (b + 1)) & 1u) f(4 * g + 1, (uint32_t)q[1]);
                if ((w >> (b + 2)) & 1u) f(4 * g + 2, (uint32_t)q[2]);
                if ((w >> (b + 3)) & 1u) f(4 * g + 3, (uint32_t)q[3]);
            }
        }
    }
};

template <>
struct MetaSrc<0> {
    const uint4 *mp;
    int T;
    __device__ __forceinline__ void init(const uint32_t *base, int tid, int TT) {
        mp = reinterpret_cast<const uint4 *>(base) + tid;
        T = TT;
    }
    template <typename F>
    __device__ __forceinline__ void each(int EPL, F &&f) const {
        const int G = (EPL + 3) >> 2;
        for (int g = 0; g < G; ++g) {
            const uint4 q = mp[(size_t)g * T];
            f(4 * g + 0, q.x);
            f(4 * g + 1, q.y);
            f(4 * g + 2, q.z);
            f(4 * g + 3, q.w);
        }
    }
};

}  // namespace dev
}  // namespace qldpc
