// trials.hip — the reference's trial generator on device.
//
// Per trial f (src/simulation.cpp:540-551): a Xoshiro256++ generator seeded
// with seeds[f] + seed_add (the simulation loop's `seeds[n] + curr_sim`,
// :743), Alice's key from uniform_int_distribution<int>(0, 1) draws
// (fill_random_bits, src/array_and_matrix_operations.cpp:889-901), Bob's key
// with exactly floor(n*QBER) errors at the first positions of a std::shuffle'd
// index vector (inject_errors, :904-933).  Draw consumption follows libstdc++
// 11 exactly: uniform_int_distribution downscales a 64-bit generator with
// Lemire's nearly-divisionless method (_S_nd over unsigned __int128), and
// std::shuffle takes the two-swaps-per-draw path (__gen_two_uniform_ints)
// because (2^64-1)/n >= n.
//
// Draws are sequential per trial, so each LANE runs one trial's generator
// chain (64 trials per wave, their state in VGPRs, every lane taking the same
// control flow: the shuffle's loop positions are the same for all trials).
// inject_errors reads only the first k = floor(n*QBER) positions of the
// shuffled index vector, and libstdc++'s std::shuffle is the forward
// Fisher-Yates whose step at position i >= 1 swaps a[i] — still i, untouched
// by the earlier steps — with some a[j], j <= i.  So positions >= k never need
// storing: a step at i >= k only writes a[j] = i when j < k, and only the
// steps at i < k swap inside the k-entry prefix.  Per-trial words (Alice's
// bits, the flips, the prefix, the punctured draws) live in a global
// workspace interleaved [word][lane] (a wave's access to one word index is one
// 256-byte line); a second kernel expands them into the byte keys, one
// workgroup per trial.  The same draws are consumed in the same order, so the
// keys are the reference's bit for bit.
//
// Two waves per 64 trials: Alice's n draws and the rest of the chain are two
// independent stretches of one generator stream, and Xoshiro256's state
// transition is linear over GF(2), so the state at draw n is J_n · s with the
// 256 x 256 bit matrix J_n = M^n (built on the host once per n).  One wave
// draws Alice's bits from s, the other starts at J_n · s and runs the shuffle
// and the punctured draws: the same draws in the same order, in parallel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <utility>

namespace qldpc {
namespace {

struct Xoshiro256pp {
    uint64_t s0, s1, s2, s3;
    __device__ static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    __device__ explicit Xoshiro256pp(uint64_t seed) {  // Xoshiro-cpp: four SplitMix64 outputs
        uint64_t x = seed;
        uint64_t *st[4] = {&s0, &s1, &s2, &s3};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint64_t z = (x += 0x9e3779b97f4a7c15ull);
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
            *st[i] = z ^ (z >> 31);
        }
    }
    __device__ uint64_t next() {
        const uint64_t r = rotl(s0 + s3, 23) + s0;
        const uint64_t t = s1 << 17;
        s2 ^= s0;
        s3 ^= s1;
        s1 ^= s2;
        s0 ^= s3;
        s2 ^= t;
        s3 = rotl(s3, 45);
        return r;
    }
};

// libstdc++ uniform_int_distribution::_S_nd<unsigned __int128>: a value in
// [0, range) from a 64-bit generator.
__device__ inline uint64_t draw_below(Xoshiro256pp &g, uint64_t range) {
    uint64_t x = g.next();
    uint64_t lo = x * range;
    uint64_t hi = __umul64hi(x, range);
    if (lo < range) {
        const uint64_t threshold = (0 - range) % range;
        while (lo < threshold) {
            x = g.next();
            lo = x * range;
            hi = __umul64hi(x, range);
        }
    }
    return hi;
}

// Words of one trial's workspace column: Alice's bits, the flips, the
// k-prefix and the punctured draws (Alice's, Bob's) as bit words.
struct TrialWs {
    int words, k, pwords;
    __host__ __device__ TrialWs(int n, uint64_t n_err, int n_punct)
        : words((n + 31) / 32), k((int)n_err), pwords((n_punct + 31) / 32) {}
    __host__ __device__ size_t per_lane() const { return 2 * (size_t)words + (size_t)k + 2 * (size_t)pwords; }
    __host__ __device__ size_t abits() const { return 0; }
    __host__ __device__ size_t flips() const { return (size_t)words; }
    __host__ __device__ size_t perm() const { return 2 * (size_t)words; }
    __host__ __device__ size_t palice() const { return 2 * (size_t)words + (size_t)k; }
    __host__ __device__ size_t pbob() const { return 2 * (size_t)words + (size_t)k + (size_t)pwords; }
};

// jump: J_n as 256 columns of four words (nullptr: one wave runs the whole
// chain); the grid then has two waves per 64 trials, Alice's bits in the first
// half of the blocks, the rest of the chain in the second.
__global__ void __launch_bounds__(64) trials_lanes_kernel(int n, uint64_t n_err, int batch, const uint64_t *seeds,
                                                          uint64_t seed_add, uint32_t *ws, int n_punct,
                                                          const uint64_t *__restrict__ jump) {
    const int lane = threadIdx.x;
    const int nblk = (batch + 63) / 64;
    const bool split = jump != nullptr;
    const bool tail = split && (int)blockIdx.x >= nblk;  // this wave starts at draw n
    const int blk = tail ? (int)blockIdx.x - nblk : (int)blockIdx.x;
    const int f = blk * 64 + lane;
    const TrialWs L(n, n_err, n_punct);
    // this wave's 64 columns, [word][lane]
    uint32_t *col = ws + (size_t)blk * L.per_lane() * 64 + lane;
    auto at = [&](size_t word) -> uint32_t & { return col[word * 64]; };
    Xoshiro256pp g((f < batch ? seeds[f] : 0ull) + seed_add);
    if (!tail) {
        // fill_random_bits: uniform_int_distribution<int>(0, 1) -> _S_nd(g, 2),
        // which never rejects: the top bit of each draw.
        for (int w = 0; w < L.words; ++w) {
            uint32_t v = 0;
            const int nb = (n - 32 * w < 32) ? n - 32 * w : 32;
            for (int b = 0; b < nb; ++b) v |= (uint32_t)(g.next() >> 63) << b;
            at(L.abits() + w) = v;
        }
        if (split) return;
    } else {
        // the state after Alice's n draws: J_n · s over GF(2) (columns by
        // wave-uniform loads)
        const uint64_t s[4] = {g.s0, g.s1, g.s2, g.s3};
        uint64_t r[4] = {0, 0, 0, 0};
        for (int j = 0; j < 256; ++j) {
            const uint64_t m = 0ull - ((s[j >> 6] >> (j & 63)) & 1ull);
#pragma unroll
            for (int q = 0; q < 4; ++q) r[q] ^= jump[4 * j + q] & m;
        }
        g.s0 = r[0];
        g.s1 = r[1];
        g.s2 = r[2];
        g.s3 = r[3];
    }
    for (int w = 0; w < L.words; ++w) at(L.flips() + w) = 0u;
    const uint32_t k = (uint32_t)n_err;
    if (k > 0) {
        for (uint32_t e = 0; e < k; ++e) at(L.perm() + e) = e;
        // one swap of std::shuffle, a[pos] <-> a[p] (p <= pos), on the k-prefix
        auto swap_at = [&](uint32_t pos, uint32_t p) {
            if (pos < k) {  // (pos is the same on every lane)
                const uint32_t t = at(L.perm() + pos), u = at(L.perm() + p);
                at(L.perm() + pos) = u;
                at(L.perm() + p) = t;
            } else if (p < k) {
                at(L.perm() + p) = pos;  // a[pos] == pos until its own step
            }
        };
        // std::shuffle(first, last, g), libstdc++ 11 (bits/stl_algo.h)
        uint64_t i = 1;
        if ((n & 1) == 0) {
            swap_at(1, (uint32_t)draw_below(g, 2));
            i = 2;
        }
        while (i != (uint64_t)n) {
            const uint64_t b0 = i + 1, b1 = i + 2;  // __gen_two_uniform_ints(b0, b0 + 1)
            const uint64_t x = draw_below(g, b0 * b1);
            uint64_t p1, p2;
            if (x < 0x100000000ull) {  // 32-bit divide when it fits (n <= 65535 always)
                const uint32_t x32 = (uint32_t)x, d32 = (uint32_t)b1;
                p1 = x32 / d32;
                p2 = x32 - (uint32_t)p1 * d32;
            } else {
                p1 = x / b1;
                p2 = x % b1;
            }
            swap_at((uint32_t)i, (uint32_t)p1);
            swap_at((uint32_t)i + 1, (uint32_t)p2);
            i += 2;
        }
        for (uint32_t e = 0; e < k; ++e) {  // inject_errors: flip pos[0 .. k)
            const uint32_t p = at(L.perm() + e);
            at(L.flips() + (p >> 5)) |= 1u << (p & 31);
        }
    }
    // QKD_LDPC_RATE_ADAPT continues the trial's generator: two
    // uniform_int_distribution<int>(0, 1) draws (Alice, then Bob) per
    // punctured position, in ascending position order
    // (src/qkd_ldpc_algorithm.cpp:1148-1157).
    for (int w = 0; w < L.pwords; ++w) {
        uint32_t va = 0, vb = 0;
        const int nb = (n_punct - 32 * w < 32) ? n_punct - 32 * w : 32;
        for (int b = 0; b < nb; ++b) {
            va |= (uint32_t)(g.next() >> 63) << b;
            vb |= (uint32_t)(g.next() >> 63) << b;
        }
        at(L.palice() + w) = va;
        at(L.pbob() + w) = vb;
    }
}

// The keys as bytes, one workgroup per trial: Alice's, Bob's (Alice's xor the
// flips) and the punctured draws.
__global__ void __launch_bounds__(256) trials_expand_kernel(int n, uint64_t n_err, int batch, const uint32_t *ws,
                                                            uint8_t *alice, uint8_t *bob, int n_punct,
                                                            uint8_t *punct_alice, uint8_t *punct_bob) {
    const int f = blockIdx.x;
    const TrialWs L(n, n_err, n_punct);
    const uint32_t *col = ws + (size_t)(f / 64) * L.per_lane() * 64 + (f % 64);
    auto at = [&](size_t word) { return col[word * 64]; };
    uint8_t *a = alice + (size_t)f * n;
    uint8_t *b = bob + (size_t)f * n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t av = (at(L.abits() + (i >> 5)) >> (i & 31)) & 1u;
        const uint32_t fv = (at(L.flips() + (i >> 5)) >> (i & 31)) & 1u;
        a[i] = (uint8_t)av;
        b[i] = (uint8_t)(av ^ fv);
    }
    for (int j = threadIdx.x; j < n_punct; j += blockDim.x) {
        punct_alice[(size_t)f * n_punct + j] = (uint8_t)((at(L.palice() + (j >> 5)) >> (j & 31)) & 1u);
        punct_bob[(size_t)f * n_punct + j] = (uint8_t)((at(L.pbob() + (j >> 5)) >> (j & 31)) & 1u);
    }
}

// QKD_LDPC_RATE_ADAPT's extended frame (src/qkd_ldpc_algorithm.cpp:1121-1180):
// position i is a key bit (cls 0: the next trial key bit, LLR +-log_p), a
// punctured bit (cls 1: the trial's extra draws, LLR ALMOST_ZERO = 1e-4) or a
// shortened bit (cls 2: 0 on both sides, LLR DBL_MAX); src[i] indexes the key
// or punctured draw.  Writes Alice's extended key, optionally the LLRs, the
// V2 palette form (codes 0/1 = +-log_p, 2 = 1e-4, 3 = DBL_MAX) and the Alice
// syndrome of the extended key.
__global__ void __launch_bounds__(256) build_frames_ra_kernel(int n, int m, const int32_t *ell_col,
                                                              const int32_t *row_deg, const uint8_t *cls,
                                                              const int32_t *src, int n_punct,
                                                              const uint8_t *alice, const uint8_t *bob,
                                                              const uint8_t *palice, const uint8_t *pbob,
                                                              const double *log_p, uint8_t *alice_ext, double *llr,
                                                              uint8_t *synd, uint8_t *codes, double *palette,
                                                              uint8_t *pal_ok, const int32_t *col_orig) {
    const size_t f = blockIdx.x;
    const double lp = log_p[f];
    const uint8_t *al = alice + f * (size_t)n;
    const uint8_t *bo = bob + f * (size_t)n;
    const uint8_t *pa = palice + f * (size_t)n_punct;
    (void)pbob;  // Bob's punctured draws only advance the generator (LLR = ALMOST_ZERO)
    uint8_t *ax = alice_ext + f * (size_t)n;
    auto bob_code = [&](int i) -> int {  // palette code of position i
        const int c = cls[i];
        if (c == 0) return bo[src[i]] ? 1 : 0;
        return c == 1 ? 2 : 3;
    };
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int c = cls[i];
        ax[i] = c == 0 ? al[src[i]] : (c == 1 ? pa[src[i]] : 0);
        if (llr) {
            const int code = bob_code(i);
            llr[f * (size_t)n + i] = code == 0 ? lp : code == 1 ? -lp : code == 2 ? 1e-4 : 1.7976931348623157e308;
        }
    }
    if (codes) {
        const int nc = (n + 3) / 4;
        uint8_t *cs = codes + f * (size_t)nc;
        for (int j = threadIdx.x; j < nc; j += blockDim.x) {
            int byte = 0;
            for (int q = 0; q < 4; ++q) {  // label order (col_orig)
                const int i = 4 * j + q;
                if (i < n) byte |= bob_code(col_orig ? col_orig[i] : i) << (2 * q);
            }
            cs[j] = (uint8_t)byte;
        }
        if (threadIdx.x < 4) {
            const double pv[4] = {lp, -lp, 1e-4, 1.7976931348623157e308};
            palette[f * 4 + threadIdx.x] = pv[threadIdx.x];
        }
        if (threadIdx.x == 0) pal_ok[f] = 1;
    }
    __syncthreads();  // the extended key is complete (global, this block)
    uint8_t *s = synd + f * (size_t)m;
    for (int j = threadIdx.x; j < m; j += blockDim.x) {
        int p = 0;
        const int deg = row_deg[j];
        for (int k = 0; k < deg; ++k) p ^= ax[ell_col[(size_t)k * m + j]];
        s[j] = (uint8_t)(p & 1);
    }
}

}  // namespace

hipError_t launch_build_frames_ra(int n, int m, const int32_t *ell_col, const int32_t *row_deg, const uint8_t *cls,
                                  const int32_t *src, int n_punct, int batch, const uint8_t *alice, const uint8_t *bob,
                                  const uint8_t *palice, const uint8_t *pbob, const double *log_p, uint8_t *alice_ext,
                                  double *llr, uint8_t *synd, uint8_t *codes, double *palette, uint8_t *pal_ok,
                                  const int32_t *col_orig, hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    hipLaunchKernelGGL(build_frames_ra_kernel, dim3(batch), dim3(256), 0, stream, n, m, ell_col, row_deg, cls, src,
                       n_punct, alice, bob, palice, pbob, log_p, alice_ext, llr, synd, codes, palette, pal_ok,
                       col_orig);
    return hipGetLastError();
}

namespace {

// J_d = M^d for Xoshiro256's state transition M, column-major: column j (four
// words) is J_d applied to the unit state e_j.  Host code, once per d.
void xo_step(uint64_t s[4]) {
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = (s[3] << 45) | (s[3] >> 19);
}
void gf2_mul(const uint64_t *A, const uint64_t *B, uint64_t *C) {  // C = A B (256 x 256, columns)
    for (int j = 0; j < 256; ++j) {
        uint64_t r[4] = {0, 0, 0, 0};
        for (int i = 0; i < 256; ++i)
            if ((B[4 * j + (i >> 6)] >> (i & 63)) & 1ull)
                for (int q = 0; q < 4; ++q) r[q] ^= A[4 * i + q];
        std::memcpy(C + 4 * j, r, sizeof r);
    }
}
void xo_jump_matrix(uint64_t d, uint64_t *J) {
    uint64_t M[1024], P[1024], T[1024];  // (24 KiB of host stack; no shared state)
    for (int j = 0; j < 256; ++j) {
        uint64_t s[4] = {0, 0, 0, 0};
        s[j >> 6] = 1ull << (j & 63);
        xo_step(s);
        std::memcpy(M + 4 * j, s, sizeof s);
    }
    std::memset(J, 0, 1024 * sizeof(uint64_t));
    for (int j = 0; j < 256; ++j) J[4 * j + (j >> 6)] = 1ull << (j & 63);
    std::memcpy(P, M, sizeof M);
    for (; d; d >>= 1) {  // powers of M commute: the product order is free
        if (d & 1) {
            gf2_mul(P, J, T);
            std::memcpy(J, T, sizeof T);
        }
        if (d > 1) {
            gf2_mul(P, P, T);
            std::memcpy(P, T, sizeof T);
        }
    }
}
// J_n on a device, built and uploaded once per (device, n) for the process.
std::mutex g_jump_mu;
std::map<std::pair<int, int>, uint64_t *> g_jump;
hipError_t jump_on_device(int n, const uint64_t **out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_jump_mu);
    auto it = g_jump.find({dev, n});
    if (it == g_jump.end()) {
        uint64_t J[1024];
        xo_jump_matrix((uint64_t)n, J);
        uint64_t *d = nullptr;
        if ((e = hipMalloc(&d, sizeof J)) != hipSuccess) return e;
        if ((e = hipMemcpy(d, J, sizeof J, hipMemcpyHostToDevice)) != hipSuccess) {
            (void)hipFree(d);
            return e;
        }
        it = g_jump.emplace(std::make_pair(dev, n), d).first;
    }
    *out = it->second;
    return hipSuccess;
}

}  // namespace

int xoshiro_jump_check(uint64_t seed, uint64_t d, uint64_t *state_out) {
    uint64_t J[1024], s[4], x = seed;
    for (auto &v : s) {  // Xoshiro-cpp seeding (four SplitMix64 outputs)
        uint64_t z = (x += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        v = z ^ (z >> 31);
    }
    xo_jump_matrix(d, J);
    for (int q = 0; q < 4; ++q) state_out[q] = 0;
    for (int j = 0; j < 256; ++j)
        if ((s[j >> 6] >> (j & 63)) & 1ull)
            for (int q = 0; q < 4; ++q) state_out[q] ^= J[4 * j + q];
    return 0;
}

size_t trials_scratch_words(int n, uint64_t n_err, int n_punct, int batch) {
    return TrialWs(n, n_err, n_punct).per_lane() * 64 * (size_t)((batch + 63) / 64);
}

hipError_t launch_trials(int n, uint64_t n_err, int batch, const uint64_t *seeds, uint64_t seed_add, uint8_t *alice,
                         uint8_t *bob, uint32_t *scratch, int n_punct, uint8_t *punct_alice, uint8_t *punct_bob,
                         hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    if (!scratch) return hipErrorInvalidValue;
    // two waves per 64 trials (QLDPC_TRIAL_SPLIT=0: one, A/B)
    const uint64_t *jump = nullptr;
    const char *env = std::getenv("QLDPC_TRIAL_SPLIT");
    if (!(env && std::strcmp(env, "0") == 0)) {
        hipError_t je = jump_on_device(n, &jump);
        if (je != hipSuccess) return je;
    }
    const int nblk = (batch + 63) / 64;
    hipLaunchKernelGGL(trials_lanes_kernel, dim3(jump ? 2 * nblk : nblk), dim3(64), 0, stream, n, n_err, batch,
                       seeds, seed_add, scratch, n_punct, jump);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(trials_expand_kernel, dim3(batch), dim3(256), 0, stream, n, n_err, batch, scratch, alice, bob,
                       n_punct, punct_alice, punct_bob);
    return hipGetLastError();
}

}  // namespace qldpc
