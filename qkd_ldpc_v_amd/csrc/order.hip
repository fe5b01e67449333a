// order.hip — the order in which the persistent decoders claim frames.
//
// The decoders pull frames from an atomic counter, one frame per workgroup at
// a time (decoder.hip, decoder_v2.hip).  Frame lengths vary a lot (C2 SPA:
// median 14 iterations, 1% of the frames run the full 50), so a batch claimed
// in index order ends with a tail in which a few long frames keep a few CUs
// busy while the rest idle (simulated on 4096 oracle-decoded C2 frames over
// 256 CUs: makespan 1.15x the ideal).
//
// Predictor: the weight of the channel decision's syndrome mismatch,
// w = |H * z XOR s|, z_i = (llr_i <= 0) — the reference's hard decision
// (src/qkd_ldpc_algorithm.cpp:80-83) on the a-priori LLRs it builds at
// :1043-1049.  Every frame the reference generates carries exactly
// floor(n * QBER) errors (src/array_and_matrix_operations.cpp:905-933), so a
// LOW weight means errors that pair up inside checks and hide from the
// syndrome: those frames decode slowest (C2 SPA: correlation -0.58 between w
// and the iteration count; every 50-iteration frame of the sample lies in the
// lowest 22% of w).  Claiming frames in ascending w is a longest-first
// schedule: simulated makespan 1.02x the ideal.
//
// The order only decides WHEN a frame is decoded; each frame's outputs are
// written at its own index, so results are identical in any order.
#include "decoder_common.hpp"

namespace qldpc {

namespace {

constexpr int ORDER_BUCKETS = 4096;  // counting-sort keys: w - min(w), clamped
constexpr int ORDER_THREADS = 1024;

// One workgroup per frame: the frame's channel decisions as a bit mask in LDS,
// then each row's parity of them against its target syndrome bit.
__global__ void __launch_bounds__(1024) frame_weight_kernel(int n, int m, const int32_t *ell_col,
                                                           const int32_t *row_deg, const uint8_t *synd,
                                                           const double *llr, const uint8_t *codes,
                                                           const double *palette, const uint8_t *pal_ok,
                                                           const int32_t *col_orig, int32_t *weight) {
    extern __shared__ uint32_t zmask[];
    const size_t f = blockIdx.x;
    const int nw = (n + 31) / 32;
    const bool pal = codes && pal_ok[f];
    double pv[4] = {0., 0., 0., 0.};
    if (pal)
        for (int q = 0; q < 4; ++q) pv[q] = palette[f * 4 + q];
    const int nc = (n + 3) / 4;
    for (int wd = threadIdx.x; wd < nw; wd += blockDim.x) {
        uint32_t z = 0;
        if (pal) {
            const uint8_t *cs = codes + f * (size_t)nc + (size_t)wd * 8;
            for (int b = 0; b < 8; ++b) {
                if (wd * 32 + 4 * b >= n) break;
                const uint32_t c = cs[b];
                for (int s = 0; s < 4; ++s) {
                    const int i = wd * 32 + 4 * b + s;
                    if (i < n && pv[(c >> (2 * s)) & 3u] <= 0.0) z |= 1u << (4 * b + s);
                }
            }
        } else {
            const double *l = llr + f * (size_t)n;
            for (int s = 0; s < 32; ++s) {
                const int i = wd * 32 + s;
                if (i < n && l[col_orig ? col_orig[i] : i] <= 0.0) z |= 1u << s;  // (bit i of z: label i)
            }
        }
        zmask[wd] = z;
    }
    __syncthreads();
    const uint8_t *sy = synd + f * (size_t)m;
    int cnt = 0;
    for (int j = threadIdx.x; j < m; j += blockDim.x)
        cnt += (int)((sy[j] & 1u) ^ dev::row_parity(zmask, ell_col, row_deg, m, j));
    // block sum
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    __shared__ int wsum[16];
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < (int)blockDim.x / 64; ++w) t += wsum[w];
        weight[f] = t;
    }
}

// One workgroup: counting sort of the frames by ascending weight (ties in any
// order — the schedule, never the results, depends on it).
__global__ void __launch_bounds__(ORDER_THREADS) frame_order_kernel(int batch, const int32_t *weight,
                                                                    int32_t *order) {
    __shared__ int hist[ORDER_BUCKETS];
    __shared__ int wmin_s;
    __shared__ int part[ORDER_THREADS / 64];
    const int tid = threadIdx.x;
    int wmin = 0x7fffffff;
    for (int f = tid; f < batch; f += ORDER_THREADS) wmin = min(wmin, weight[f]);
    for (int o = 32; o > 0; o >>= 1) wmin = min(wmin, __shfl_xor(wmin, o, 64));
    if (tid == 0) wmin_s = 0x7fffffff;
    for (int i = tid; i < ORDER_BUCKETS; i += ORDER_THREADS) hist[i] = 0;
    __syncthreads();
    if ((tid & 63) == 0) atomicMin(&wmin_s, wmin);
    __syncthreads();
    wmin = wmin_s;
    auto key = [&](int f) { return min(weight[f] - wmin, ORDER_BUCKETS - 1); };
    for (int f = tid; f < batch; f += ORDER_THREADS) atomicAdd(&hist[key(f)], 1);
    __syncthreads();
    // exclusive scan of the histogram: 4 buckets per thread, then across threads
    constexpr int PER = ORDER_BUCKETS / ORDER_THREADS;
    int loc[PER], s = 0;
    for (int i = 0; i < PER; ++i) {
        loc[i] = s;
        s += hist[tid * PER + i];
    }
    int incl = s;  // inclusive scan of s over the block
    const int lane = tid & 63;
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) part[tid >> 6] = incl;
    __syncthreads();
    int base = incl - s;
    for (int w = 0; w < (tid >> 6); ++w) base += part[w];
    __syncthreads();
    for (int i = 0; i < PER; ++i) hist[tid * PER + i] = base + loc[i];
    __syncthreads();
    for (int f = tid; f < batch; f += ORDER_THREADS) order[atomicAdd(&hist[key(f)], 1)] = f;
}

}  // namespace

size_t frame_weight_lds(int n) { return (size_t)((n + 31) / 32) * 4; }

hipError_t launch_frame_order(int n, int m, const int32_t *ell_col, const int32_t *row_deg, int batch,
                              const uint8_t *synd, const double *llr, const uint8_t *codes,
                              const double *palette, const uint8_t *pal_ok, int32_t *weight, int32_t *order,
                              const int32_t *col_orig, hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    // (n near 2^20 needs up to 128 KiB of dynamic LDS: opt in like every large-LDS launch)
    hipError_t ea = allow_dynamic_lds(reinterpret_cast<const void *>(frame_weight_kernel), frame_weight_lds(n));
    if (ea != hipSuccess) return ea;
    hipLaunchKernelGGL(frame_weight_kernel, dim3(batch), dim3(aux_frame_threads(n)), frame_weight_lds(n), stream, n, m, ell_col,
                       row_deg, synd, llr, codes, palette, pal_ok, col_orig, weight);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(frame_order_kernel, dim3(1), dim3(ORDER_THREADS), 0, stream, batch, weight, order);
    return hipGetLastError();
}

}  // namespace qldpc
