// valu_bench.hip — FP64 VALU ceilings of the SPA edge update on gfx950.
//
// Measures, with no memory traffic in the timed loops:
//   fma      independent v_fma_f64 chains            (peak f64 VALU rate)
//   rcp      v_rcp_f64 chains                         (transcendental rate)
//   div      IEEE f64 division                        (div_scale/rcp/fma/fixup)
//   edge     tanh_dec(x/2) -> p/t -> 2*atanh_dec()    (one SPA edge, math only)
// and prints one JSON line.  Build: make valu_bench; run on the GPU box.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../qkd_ldpc_v_amd/csrc/exact_math.h"

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
            return 1;                                                             \
        }                                                                         \
    } while (0)

constexpr int CH = 8;

__global__ void __launch_bounds__(256) k_fma(int iters, double *out) {
    double v[CH];
    for (int c = 0; c < CH; ++c) v[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) v[c] = __builtin_fma(v[c], 0.999999, 1e-7);
    double s = 0;
    for (int c = 0; c < CH; ++c) s += v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__device__ unsigned long long g_cycles;

__global__ void __launch_bounds__(256) k_fma_clk(int iters, double *out) {
    const unsigned long long c0 = clock64();
    double v[CH];
    for (int c = 0; c < CH; ++c) v[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) v[c] = __builtin_fma(v[c], 0.999999, 1e-7);
    double s = 0;
    for (int c = 0; c < CH; ++c) s += v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (blockIdx.x == 0 && threadIdx.x == 0) g_cycles = clock64() - c0;
}

__global__ void __launch_bounds__(256) k_int(int iters, double *out) {
    uint32_t v[CH];
    for (int c = 0; c < CH; ++c) v[c] = threadIdx.x * 7 + c;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) v[c] = (v[c] ^ 0x9e3779b9u) + (uint32_t)c;
    double s = 0;
    for (int c = 0; c < CH; ++c) s += v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_sel(int iters, double *out) {
    double v[CH];
    for (int c = 0; c < CH; ++c) v[c] = threadIdx.x * 1e-3 + c;
    const double a = out[0], b = out[1];
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            asm volatile("" : "+v"(v[c]));
            v[c] = (v[c] > 1.0) ? a : v[c] + b;
        }
    double s = 0;
    for (int c = 0; c < CH; ++c) s += v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_rcp(int iters, double *out) {
    double v[CH];
    for (int c = 0; c < CH; ++c) v[c] = 1.0 + threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) v[c] = __builtin_amdgcn_rcp(v[c]);
    double s = 0;
    for (int c = 0; c < CH; ++c) s += v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_div(int iters, double *out) {
    double v[CH];
    for (int c = 0; c < CH; ++c) v[c] = 1.0 + threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) v[c] = 3.0 / v[c];
    double s = 0;
    for (int c = 0; c < CH; ++c) s += v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

constexpr int ECH = 2;
__global__ void __launch_bounds__(256) k_edge(int iters, double *out) {
    double x[ECH];
    for (int c = 0; c < ECH; ++c) x[c] = (threadIdx.x % 97) * 0.37 - 18.0 + c;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int c = 0; c < ECH; ++c) {
            const double t = ql_exact::tanh_dec(x[c] / 2.);
            const double p = (t * 0.7) / t;
            x[c] = 2. * ql_exact::atanh_dec(p * 0.9) + (c ? 0.25 : -0.25);
        }
    double s = 0;
    for (int c = 0; c < ECH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
float timeit(K kern, int blocks, int iters, double *out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, iters / 8, out);  // warm
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, iters, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    int cus = 0, clk = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
    const int blocks = cus * 8;  // 8 x 256 threads = 32 waves per CU (8 per SIMD)
    double *out;
    CK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(double)));
    const double lanes = (double)blocks * 256;
    const int it = 20000, ite = 400;
    const float t_fma = timeit(k_fma, blocks, it, out);
    const float t_rcp = timeit(k_rcp, blocks, it, out);
    const float t_div = timeit(k_div, blocks, it / 4, out);
    const float t_edge = timeit(k_edge, blocks, ite, out);
    const float t_clk = timeit(k_fma_clk, blocks, it, out);
    const float t_int = timeit(k_int, blocks, it, out);
    const float t_sel = timeit(k_sel, blocks, it, out);
    CK(hipDeviceSynchronize());
    unsigned long long cyc = 0;
    CK(hipMemcpyFromSymbol(&cyc, HIP_SYMBOL(g_cycles), sizeof(cyc)));
    // per-lane operations per second
    const double fma_s = lanes * it * CH / (t_fma * 1e-3);
    const double rcp_s = lanes * it * CH / (t_rcp * 1e-3);
    const double div_s = lanes * (it / 4) * CH / (t_div * 1e-3);
    const double edge_s = lanes * ite * ECH / (t_edge * 1e-3);
    // int: one v_xad_u32 per step; sel: cmp_f64 + add_f64 + 2 cndmask per step (wave-instructions)
    const double wi = lanes / 64.0 * it * CH;
    printf("{\"fma_clk_ms\": %.3f, \"wave_cycles_fma\": %llu, \"int32_wave_instr_per_s\": %.4e, "
           "\"sel_step_per_s\": %.4e, \"fma_wave_instr_per_s\": %.4e}\n",
           t_clk, cyc, wi / (t_int * 1e-3), wi / (t_sel * 1e-3), wi / (t_clk * 1e-3));
    printf("{\"cus\": %d, \"clock_khz\": %d, \"fma_f64_lane_ops_per_s\": %.4e, \"fma_tflops\": %.2f, "
           "\"rcp_f64_lane_ops_per_s\": %.4e, \"div_f64_lane_ops_per_s\": %.4e, "
           "\"spa_edge_math_per_s\": %.4e, \"ms\": [%.3f, %.3f, %.3f, %.3f]}\n",
           cus, clk, fma_s, 2 * fma_s / 1e12, rcp_s, div_s, edge_s, t_fma, t_rcp, t_div, t_edge);
    return 0;
}
