// trials.hip — the reference's trial generator on device.
//
// Per trial f (src/simulation.cpp:540-551): a Xoshiro256++ generator seeded
// with seeds[f] + seed_add (the simulation loop's `seeds[n] + curr_sim`,
// :743), Alice's key from uniform_int_distribution<int>(0, 1) draws
// (fill_random_bits, src/array_and_matrix_operations.cpp:889-901), Bob's key
// with exactly k = floor(n*QBER) errors at the first positions of a
// std::shuffle'd index vector (inject_errors, :904-933), then, for
// QKD_LDPC_RATE_ADAPT, two uniform_int_distribution<int>(0, 1) draws per
// punctured position (src/qkd_ldpc_algorithm.cpp:1148-1157).  Draw consumption
// follows libstdc++ 11 exactly: uniform_int_distribution downscales a 64-bit
// generator with Lemire's nearly-divisionless method (_S_nd over unsigned
// __int128), and std::shuffle takes the two-swaps-per-draw path
// (__gen_two_uniform_ints) because (2^64-1)/n >= n.
//
// One trial's draws are one sequential stream of D = n + S + 2 n_punct
// generator outputs (S = the shuffle's draws: n/2 for even n, (n-1)/2 for odd
// n).  Xoshiro256's state transition is linear over GF(2), so the state at
// draw d is J_d · s (J_d = M^d, a 256 x 256 bit matrix): the stream is cut
// into units of kUnit draws and every segment starts from J_{u kUnit} · s (a
// host-built table, one matrix per unit index, shared by every n).  Alice's
// cheap draws go kAliceUnits units to a segment, the shuffle's and the
// punctured draws (a 64-bit product and a division each) one unit.  A wave
// runs one segment of 64 trials (one per lane: the segment's control flow
// and its matrix loads are wave-uniform), so a batch's generation is
// (batch / 64) x segments independent waves instead of 64 sequential chains
// of D draws.
//
// What each draw means is fixed by its index alone, except that a shuffle
// draw may be rejected by _S_nd (probability < range / 2^64 per draw: < 1e-9
// at n = 100k) and then shifts every later draw.  A lane that meets a
// rejection flags its trial, and the finish kernel reruns that trial's
// shuffle and punctured draws sequentially (the reference's order exactly).
//
// The shuffle: inject_errors reads only the first k positions of the shuffled
// index vector, and libstdc++'s std::shuffle is the forward Fisher-Yates whose
// step at position i >= 1 swaps a[i] — still i, untouched by the earlier
// steps — with some a[p], p <= i.  So a step at i < k is a swap inside the
// k-prefix (kept: p goes to pbuf[i]), and a step at i >= k only writes
// a[p] = i when p < k — the LAST such write wins, i.e. the largest i, which
// the draw kernel keeps with an atomic max per prefix entry (last[p]).  The
// finish kernel resolves the k - 1 prefix swaps (below), takes last[p] where
// set, and flips Bob's key at the k resulting positions.  The same draws are
// consumed in the same order: the keys are the reference's bit for bit.
//
// The prefix swaps are the inside-out shuffle: step i puts the value i at p_i
// and moves the old a[p_i] to i.  So position x ends holding the last step
// i > x with p_i = x (a "writer" of x) if there is one; otherwise the value
// its own step x moved in, i.e. what position p_x held just before step x —
// the last writer of p_x below x, or failing one, what p_x's own step moved
// in, and so on down a chain of decreasing positions (x = 0, or a step with
// p_y = y, ends it with the position itself).  With every position's writers
// listed, each prefix position is resolved independently: the finish kernel
// walks the k chains in parallel (expected chain length O(log k)) instead of
// replaying k - 1 dependent LDS swaps on one thread.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "decoder_common.hpp"

#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

namespace qldpc {
namespace {

constexpr int kUnit = 128;      // draws per jump-table unit (one wave runs one segment of 64 trials)
constexpr int kAliceUnits = 4;  // units per segment in Alice's part of the stream
constexpr uint32_t kPrefixLds = 16384;  // k-prefix entries the finish kernel keeps in LDS (a and p: 128 KiB)
constexpr uint32_t kParLds = 12288;     // ... for the parallel replay (p, writer lists: 3k + 1 words, 144 KiB)

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
// [0, range) from a 64-bit generator (the rejection loop included).
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

// (x / b1, x % b1) of __gen_two_uniform_ints, x < b1 (b1 - 1).
// b1 < 2^20 (n < 2^20 - 2): an f32 estimate — x and 1 / b1 each within 2^-23
// relative, the product within 3e-7, so for a quotient below 2^20 the
// truncated estimate is off by at most one — corrected by the remainder's
// sign and size.  Otherwise, for x < 2^51 the quotient through f64 is exact:
// x and b1 are exact doubles, and when x / b1 is not an integer it lies at
// least 1 / b1 below the next integer N + 1, more than half an ulp of
// N + 1 < 2^52 / b1 (b1 (N + 1) <= x + b1 < 2^52), so the correctly rounded
// quotient truncates to floor(x / b1).  Beyond that, integer division.
__device__ inline void split_two(uint64_t x, uint64_t b1, uint64_t &p1, uint64_t &p2) {
    if (b1 < (1ull << 20)) {
        const float xf = __builtin_fmaf((float)(uint32_t)(x >> 32), 4294967296.0f, (float)(uint32_t)x);
        const float qf = xf * __builtin_amdgcn_rcpf((float)(uint32_t)b1);
        int64_t q = (int64_t)(uint32_t)qf;
        int64_t r = (int64_t)x - q * (int64_t)b1;
        if (r < 0) {
            --q;
            r += (int64_t)b1;
        } else if (r >= (int64_t)b1) {
            ++q;
            r -= (int64_t)b1;
        }
        p1 = (uint64_t)q;
        p2 = (uint64_t)r;
        return;
    }
    if (x < (1ull << 51)) {
        p1 = (uint64_t)((double)x / (double)b1);
    } else {
        p1 = x / b1;
    }
    p2 = x - p1 * b1;
}

// One trial's draw stream: [0, n) Alice's bits, [n, n + S) the shuffle,
// [n + S, D) the punctured draws (Alice's, Bob's per position).  Segments:
// units [0, ceil(n / kUnit)) in groups of kAliceUnits (the last group may
// reach into the shuffle), then one unit each.
struct TrialStream {
    uint64_t n, S, D, units, aseg;
    __host__ __device__ TrialStream(int n_, int n_punct)
        : n((uint64_t)n_), S((n_ % 2 == 0) ? (uint64_t)n_ / 2 : (uint64_t)(n_ - 1) / 2),
          D((uint64_t)n_ + S + 2 * (uint64_t)n_punct), units((D + kUnit - 1) / kUnit),
          aseg(((n + kUnit - 1) / kUnit + kAliceUnits - 1) / kAliceUnits) {}
    __host__ __device__ uint64_t segments() const {
        const uint64_t au = aseg * kAliceUnits < units ? aseg * kAliceUnits : units;
        return aseg + (units - au);
    }
    // first and one-past-last unit of segment j
    __host__ __device__ void seg_units(uint64_t j, uint64_t &u0, uint64_t &u1) const {
        if (j < aseg) {
            u0 = j * kAliceUnits;
            u1 = u0 + kAliceUnits;
        } else {
            u0 = aseg * kAliceUnits + (j - aseg);
            u1 = u0 + 1;
        }
        if (u1 > units) u1 = units;
    }
};

// Generator workspace, uint32 words, BP = batch rounded up to 64:
// pbuf [k][BP] (prefix swap partner of position i < k), last [BP][k] (largest
// i >= k that wrote prefix entry p; 0 = none), abuf [BP][k] (the prefix when
// it exceeds LDS), flag [BP] (a rejected shuffle draw: rerun serially).
struct TrialWs {
    size_t k, BP;
    __host__ __device__ TrialWs(uint64_t k_, int batch) : k((size_t)k_), BP(((size_t)batch + 63) / 64 * 64) {}
    __host__ __device__ size_t pbuf() const { return 0; }
    __host__ __device__ size_t last() const { return k * BP; }
    __host__ __device__ size_t abuf() const { return 2 * k * BP; }
    __host__ __device__ size_t flag() const { return 3 * k * BP; }
    __host__ __device__ size_t words() const { return 3 * k * BP + BP; }
};

// Draw kernel: block (segment j, trial group of 64), one lane per trial.
__global__ void __launch_bounds__(64) trials_draw_kernel(int n, uint32_t k, int n_punct, int batch,
                                                         const uint64_t *__restrict__ seeds, uint64_t seed_add,
                                                         const uint64_t *__restrict__ jt, int wide,
                                                         uint8_t *__restrict__ alice, uint8_t *__restrict__ bob,
                                                         uint8_t *__restrict__ palice, uint8_t *__restrict__ pbob,
                                                         uint32_t *__restrict__ ws) {
    const int lane = threadIdx.x;
    const int f = (int)blockIdx.y * 64 + lane;
    const bool act = f < batch;
    const TrialStream T(n, n_punct);
    const TrialWs W(k, batch);
    uint64_t u0, u1;
    T.seg_units(blockIdx.x, u0, u1);
    uint64_t d = u0 * kUnit;
    const uint64_t d1 = (u1 * kUnit < T.D) ? u1 * kUnit : T.D;
    Xoshiro256pp g((act ? seeds[f] : 0ull) + seed_add);
    if (u0 > 0) {  // the state at draw u0 * kUnit: J · s over GF(2)
        // the segment's matrix (8 KiB) staged in LDS by one coalesced load round
        // (eight 16-byte loads per lane in flight), then its columns read by
        // broadcast LDS reads
        __shared__ uint4 jl[512];
        const uint4 *J4 = reinterpret_cast<const uint4 *>(jt + u0 * 1024);
        uint4 v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = J4[q * 64 + lane];
#pragma unroll
        for (int q = 0; q < 8; ++q) jl[q * 64 + lane] = v[q];
        __syncthreads();
        const uint64_t st[4] = {g.s0, g.s1, g.s2, g.s3};
        uint64_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint64_t sw = st[w];
#pragma unroll 8
            for (int b = 0; b < 64; ++b) {
                const uint64_t m = 0ull - ((sw >> b) & 1ull);
                const uint4 c01 = jl[2 * (64 * w + b)], c23 = jl[2 * (64 * w + b) + 1];
                r0 ^= (((uint64_t)c01.y << 32) | c01.x) & m;
                r1 ^= (((uint64_t)c01.w << 32) | c01.z) & m;
                r2 ^= (((uint64_t)c23.y << 32) | c23.x) & m;
                r3 ^= (((uint64_t)c23.w << 32) | c23.z) & m;
            }
        }
        g.s0 = r0;
        g.s1 = r1;
        g.s2 = r2;
        g.s3 = r3;
    }
    // fill_random_bits: _S_nd(g, 2) never rejects — the top bit of each draw.
    // Bob's key starts as a copy of Alice's; the finish kernel flips it.
    const uint64_t ae = d1 < T.n ? d1 : T.n;
    if (d < ae) {
        uint8_t *ap = alice + (size_t)f * (size_t)n;
        uint8_t *bp = bob + (size_t)f * (size_t)n;
        if (wide) {  // n % 16 == 0 and 16-byte aligned keys: one 16-byte store per 16 draws
            for (; d < ae; d += 16) {
                uint32_t w[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t v = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) v |= (uint32_t)(g.next() >> 63) << (8 * b);
                    w[q] = v;
                }
                if (act) {
                    const uint4 v4 = make_uint4(w[0], w[1], w[2], w[3]);
                    *reinterpret_cast<uint4 *>(ap + d) = v4;
                    *reinterpret_cast<uint4 *>(bp + d) = v4;
                }
            }
        } else {
            for (; d < ae; ++d) {
                const uint8_t v = (uint8_t)(g.next() >> 63);
                if (act) {
                    ap[d] = v;
                    bp[d] = v;
                }
            }
        }
    }
    // std::shuffle (libstdc++ 11, bits/stl_algo.h), one step per position
    uint32_t *pbuf = ws + W.pbuf();
    uint32_t *last = ws + W.last() + (size_t)f * W.k;
    auto record = [&](uint64_t pos, uint64_t p) {
        if (pos < k) {  // a swap inside the prefix (pos is wave-uniform): replayed in order later
            if (act) pbuf[pos * W.BP + f] = (uint32_t)p;
        } else if (p < k && act) {  // a[p] = pos; the largest pos wins
            atomicMax(last + p, (uint32_t)pos);
        }
    };
    const uint64_t se = d1 < T.n + T.S ? d1 : T.n + T.S;
    bool rejected = false;
    for (; d < se; ++d) {
        const uint64_t t = d - T.n;
        if ((n & 1) == 0 && t == 0) {  // even n: the first swap takes a single (0, 1) draw
            record(1, g.next() >> 63);
            continue;
        }
        const uint64_t i = (n & 1) == 0 ? 2 * t : 2 * t + 1;
        const uint64_t b1 = i + 2, range = (i + 1) * b1;  // __gen_two_uniform_ints(i + 1, i + 2)
        const uint64_t x = g.next();
        const uint64_t lo = x * range;
        if (lo < range) {
            const uint64_t threshold = (0 - range) % range;
            if (lo < threshold) rejected = true;  // every later draw of this trial shifts
        }
        uint64_t p1, p2;
        split_two(__umul64hi(x, range), b1, p1, p2);
        record(i, p1);
        record(i + 1, p2);
    }
    if (rejected && act) ws[W.flag() + f] = 1u;
    // QKD_LDPC_RATE_ADAPT continues the trial's generator: Alice's then Bob's
    // draw per punctured position, in ascending position order.
    for (; d < d1; ++d) {
        const uint64_t t = d - T.n - T.S;
        const uint8_t v = (uint8_t)(g.next() >> 63);
        if (act) ((t & 1) ? pbob : palice)[(size_t)f * (size_t)n_punct + (t >> 1)] = v;
    }
}

// The parallel prefix resolution (file header), one workgroup of 256 per
// trial, k <= kParLds: p (k words), the writer lists in CSR form (offsets
// k + 1, entries k), all in LDS.
__device__ void finish_parallel(uint32_t k, int f, const TrialWs &W, const uint32_t *__restrict__ ws, uint32_t *sh,
                                const uint8_t *__restrict__ alice, uint8_t *__restrict__ bob, int n) {
    __shared__ uint32_t part[256];
    const uint32_t tid = threadIdx.x, T = blockDim.x;
    uint32_t *pl = sh, *off = sh + k, *lst = sh + 2 * k + 1;
    for (uint32_t j = tid; j < k; j += T) {
        pl[j] = j ? ws[W.pbuf() + (size_t)j * W.BP + f] : 0u;
        off[j] = 0u;
    }
    __syncthreads();
    for (uint32_t j = 1 + tid; j < k; j += T) {  // writer counts (p_j < j: j writes p_j)
        const uint32_t p = pl[j];
        if (p < j) atomicAdd(off + p, 1u);
    }
    __syncthreads();
    // inclusive scan of the counts: a contiguous chunk per thread, the 256
    // chunk sums scanned by wave 0 (four per lane)
    const uint32_t C = (k + T - 1) / T, b0 = min(k, tid * C), b1 = min(k, b0 + C);
    uint32_t sum = 0;
    for (uint32_t i = b0; i < b1; ++i) sum += off[i];
    part[tid] = sum;
    __syncthreads();
    if (tid < 64) {
        const uint32_t v0 = part[4 * tid], v1 = part[4 * tid + 1], v2 = part[4 * tid + 2], v3 = part[4 * tid + 3];
        const uint32_t tot = v0 + v1 + v2 + v3;
        uint32_t inc = tot;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(inc, d, 64);
            if ((int)tid >= d) inc += o;
        }
        const uint32_t ex = inc - tot;  // exclusive prefix of the lane's four chunks
        part[4 * tid] = ex;
        part[4 * tid + 1] = ex + v0;
        part[4 * tid + 2] = ex + v0 + v1;
        part[4 * tid + 3] = ex + v0 + v1 + v2;
    }
    __syncthreads();
    uint32_t run = part[tid];
    for (uint32_t i = b0; i < b1; ++i) {
        run += off[i];
        off[i] = run;
    }
    __syncthreads();
    if (tid == 0) off[k] = off[k - 1];  // the entry count (end of the last list)
    __syncthreads();
    // fill from the back: off[p] ends at the start of p's list
    for (uint32_t j = 1 + tid; j < k; j += T) {
        const uint32_t p = pl[j];
        if (p < j) lst[atomicSub(off + p, 1u) - 1u] = j;
    }
    __syncthreads();
    const uint32_t *last = ws + W.last() + (size_t)f * W.k;
    const uint8_t *ap = alice + (size_t)f * (size_t)n;
    uint8_t *bp = bob + (size_t)f * (size_t)n;
    for (uint32_t x = tid; x < k; x += T) {
        uint32_t cur = x, bound = k, val;
        for (;;) {
            uint32_t best = 0;  // (writers are >= 1)
            for (uint32_t q = off[cur], qe = off[cur + 1]; q < qe; ++q) {
                const uint32_t i = lst[q];
                best = (i < bound && i > best) ? i : best;
            }
            if (best) {
                val = best;
                break;
            }
            if (cur == 0) {
                val = 0;
                break;
            }
            const uint32_t p = pl[cur];
            if (p == cur) {
                val = cur;
                break;
            }
            bound = cur;
            cur = p;
        }
        const uint32_t lw = last[x];
        const uint32_t pos = lw ? lw : val;
        bp[pos] = (uint8_t)(ap[pos] ^ 1u);
    }
}

// Finish kernel, one workgroup per trial: resolve the prefix swaps, merge the
// last writers, flip Bob's key at the k chosen positions.  A trial with a
// rejected shuffle draw (or every trial under force_serial) reruns its
// shuffle and punctured draws sequentially from the state after Alice's bits.
__global__ void __launch_bounds__(256) trials_finish_kernel(int n, uint32_t k, int n_punct, int batch,
                                                            const uint64_t *__restrict__ seeds, uint64_t seed_add,
                                                            const uint8_t *__restrict__ alice,
                                                            uint8_t *__restrict__ bob, uint8_t *__restrict__ palice,
                                                            uint8_t *__restrict__ pbob, uint32_t *__restrict__ ws,
                                                            int force_serial) {
    extern __shared__ uint32_t sh[];
    const int f = blockIdx.x;
    const TrialWs W(k, batch);
    const bool serial0 = force_serial == 1 || ws[W.flag() + f] != 0u;
    if (!serial0 && k <= kParLds && force_serial != 2) {
        finish_parallel(k, f, W, ws, sh, alice, bob, n);
        return;
    }
    const bool in_lds = k <= kPrefixLds;
    uint32_t *a = in_lds ? sh : ws + W.abuf() + (size_t)f * W.k;
    uint32_t *pl = in_lds ? sh + k : nullptr;  // this trial's pbuf column, staged
    const bool serial = serial0;
    for (uint32_t j = threadIdx.x; j < k; j += blockDim.x) {
        a[j] = j;
        if (pl && !serial) pl[j] = j ? ws[W.pbuf() + (size_t)j * W.BP + f] : 0u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!serial) {
            if (pl) {
                for (uint32_t pos = 1; pos < k; ++pos) {  // a[pos] == pos until its own step
                    const uint32_t p = pl[pos];
                    const uint32_t t = a[p];
                    a[p] = pos;
                    a[pos] = t;
                }
            } else {
                for (uint32_t pos = 1; pos < k; ++pos) {
                    const uint32_t p = ws[W.pbuf() + (size_t)pos * W.BP + f];
                    const uint32_t t = a[p];
                    a[p] = pos;
                    a[pos] = t;
                }
            }
        } else {
            Xoshiro256pp g(seeds[f] + seed_add);
            for (int i = 0; i < n; ++i) (void)g.next();  // Alice's draws (already written)
            auto swap_at = [&](uint64_t pos, uint64_t p) {
                if (pos < k) {
                    const uint32_t t = a[pos], u = a[p];
                    a[pos] = u;
                    a[p] = t;
                } else if (p < k) {
                    a[p] = (uint32_t)pos;
                }
            };
            uint64_t i = 1;
            if ((n & 1) == 0) {
                swap_at(1, draw_below(g, 2));
                i = 2;
            }
            while (i != (uint64_t)n) {
                const uint64_t b1 = i + 2;
                uint64_t p1, p2;
                split_two(draw_below(g, (i + 1) * b1), b1, p1, p2);
                swap_at(i, p1);
                swap_at(i + 1, p2);
                i += 2;
            }
            for (int q = 0; q < n_punct; ++q) {
                palice[(size_t)f * n_punct + q] = (uint8_t)(g.next() >> 63);
                pbob[(size_t)f * n_punct + q] = (uint8_t)(g.next() >> 63);
            }
        }
    }
    __syncthreads();
    // inject_errors: flip Bob's key at a[0 .. k)
    const uint32_t *last = ws + W.last() + (size_t)f * W.k;
    const uint8_t *ap = alice + (size_t)f * (size_t)n;
    uint8_t *bp = bob + (size_t)f * (size_t)n;
    for (uint32_t j = threadIdx.x; j < k; j += blockDim.x) {
        const uint32_t lw = serial ? 0u : last[j];
        const uint32_t pos = lw ? lw : a[j];
        bp[pos] = (uint8_t)(ap[pos] ^ 1u);
    }
}

// QKD_LDPC_RATE_ADAPT's extended frame (src/qkd_ldpc_algorithm.cpp:1121-1180):
// position i is a key bit (cls 0: the next trial key bit, LLR +-log_p), a
// punctured bit (cls 1: the trial's extra draws, LLR ALMOST_ZERO = 1e-4) or a
// shortened bit (cls 2: 0 on both sides, LLR DBL_MAX); src[i] indexes the key
// or punctured draw.  Writes Alice's extended key, optionally the LLRs, the
// V2 palette form (codes 0/1 = +-log_p, 2 = 1e-4, 3 = DBL_MAX) and the Alice
// syndrome of the extended key.  One workgroup per frame; the keys, the
// punctured draws and the extended key live in LDS as bit words, so every
// gather (by src, by label, by row) reads LDS.
__global__ void __launch_bounds__(1024) build_frames_ra_kernel(int n, int m, const int32_t *ell_col,
                                                              const int32_t *row_deg, const uint8_t *cls,
                                                              const int32_t *src, int n_punct,
                                                              const uint8_t *alice, const uint8_t *bob,
                                                              const uint8_t *palice, const uint8_t *pbob,
                                                              const double *log_p, uint8_t *alice_ext, double *llr,
                                                              uint8_t *synd, uint8_t *codes, double *palette,
                                                              uint8_t *pal_ok, const int32_t *col_orig) {
    extern __shared__ uint32_t kb[];
    const int nw = (n + 31) / 32, pw = (n_punct + 31) / 32, xw = 2 * ((n + 63) / 64);
    uint32_t *abits = kb, *bbits = kb + nw, *pbits = kb + 2 * nw, *xbits = kb + 2 * nw + pw;
    const size_t f = blockIdx.x;
    const double lp = log_p[f];
    (void)pbob;  // Bob's punctured draws only advance the generator (LLR = ALMOST_ZERO)
    dev::pack_key_bits(alice + f * (size_t)n, n, abits);
    dev::pack_key_bits(bob + f * (size_t)n, n, bbits);
    if (n_punct > 0) dev::pack_key_bits(palice + f * (size_t)n_punct, n_punct, pbits);
    __syncthreads();
    // the extended Alice key, 64 positions per wave ballot
    const int lane = threadIdx.x & 63;
    for (int base = (int)(threadIdx.x & ~63u); base < 32 * xw; base += blockDim.x) {
        const int i = base + lane;
        uint32_t bit = 0;
        if (i < n) {
            const int c = cls[i];
            bit = c == 0 ? dev::key_bit(abits, src[i]) : (c == 1 ? dev::key_bit(pbits, src[i]) : 0u);
        }
        const uint64_t bal = __ballot(bit);
        if (lane == 0) {
            xbits[base >> 5] = (uint32_t)bal;
            xbits[(base >> 5) + 1] = (uint32_t)(bal >> 32);
        }
    }
    __syncthreads();
    auto bob_code = [&](int i) -> int {  // palette code of position i
        const int c = cls[i];
        if (c == 0) return (int)dev::key_bit(bbits, src[i]);
        return c == 1 ? 2 : 3;
    };
    uint8_t *ax = alice_ext + f * (size_t)n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        ax[i] = (uint8_t)dev::key_bit(xbits, i);
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
    uint8_t *s = synd + f * (size_t)m;
    for (int j = threadIdx.x; j < m; j += blockDim.x) s[j] = (uint8_t)dev::row_parity(xbits, ell_col, row_deg, m, j);
}

}  // namespace

hipError_t launch_build_frames_ra(int n, int m, const int32_t *ell_col, const int32_t *row_deg, const uint8_t *cls,
                                  const int32_t *src, int n_punct, int batch, const uint8_t *alice, const uint8_t *bob,
                                  const uint8_t *palice, const uint8_t *pbob, const double *log_p, uint8_t *alice_ext,
                                  double *llr, uint8_t *synd, uint8_t *codes, double *palette, uint8_t *pal_ok,
                                  const int32_t *col_orig, hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    // LDS: Alice's and Bob's keys, the punctured draws and the extended key as bit words
    const size_t lds = build_frames_ra_lds(n, n_punct);
    if (lds > LDS_MAX_BYTES) return hipErrorInvalidValue;
    if (lds > 65536) {
        hipError_t e = allow_dynamic_lds(reinterpret_cast<const void *>(build_frames_ra_kernel), lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(build_frames_ra_kernel, dim3(batch), dim3(aux_frame_threads(n)), lds, stream, n, m, ell_col, row_deg, cls,
                       src, n_punct, alice, bob, palice, pbob, log_p, alice_ext, llr, synd, codes, palette, pal_ok,
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

namespace {

// Jump tables: entry j = J_{j kUnit} (column-major, 1024 words), entry 0 the
// identity, entry j + 1 = J_kUnit · entry j by four-Russians tables of J_kUnit
// (32 byte-groups x 256 column combinations).  One table per device, shared by
// every n; it grows to the longest stream asked for and is never freed (a
// retired shorter copy may still be read by a launch in flight).
struct JumpTable {
    std::vector<uint64_t> host;  // entries x 1024 words
    uint64_t *dev = nullptr;
    size_t dev_entries = 0;
};
std::mutex g_jt_mu;
std::map<int, JumpTable> g_jt;
std::vector<uint64_t> g_jt_host;  // host entries, shared by the devices
std::vector<uint64_t> g_jl_russ;  // J_kUnit as 32 x 256 column combinations (4 words each)

void jt_extend_host(size_t entries) {  // (g_jt_mu held)
    if (g_jt_host.empty()) {
        uint64_t I[1024];
        xo_jump_matrix(0, I);
        g_jt_host.assign(I, I + 1024);
        uint64_t J[1024];
        xo_jump_matrix((uint64_t)kUnit, J);
        g_jl_russ.assign(32 * 256 * 4, 0);
        for (int grp = 0; grp < 32; ++grp)
            for (int b = 1; b < 256; ++b) {
                const int low = __builtin_ctz((unsigned)b);
                const uint64_t *prev = &g_jl_russ[((size_t)grp * 256 + (b & (b - 1))) * 4];
                const uint64_t *col = J + 4 * (8 * grp + low);
                uint64_t *dst = &g_jl_russ[((size_t)grp * 256 + b) * 4];
                for (int q = 0; q < 4; ++q) dst[q] = prev[q] ^ col[q];
            }
    }
    while (g_jt_host.size() / 1024 < entries) {
        const uint64_t *B = &g_jt_host[g_jt_host.size() - 1024];
        uint64_t C[1024];
        for (int c = 0; c < 256; ++c) {  // column c of J_kUnit · B
            uint64_t r[4] = {0, 0, 0, 0};
            for (int grp = 0; grp < 32; ++grp) {
                const unsigned byte = (unsigned)(B[4 * c + grp / 8] >> (8 * (grp % 8))) & 0xffu;
                const uint64_t *t = &g_jl_russ[((size_t)grp * 256 + byte) * 4];
                for (int q = 0; q < 4; ++q) r[q] ^= t[q];
            }
            std::memcpy(C + 4 * c, r, sizeof r);
        }
        g_jt_host.insert(g_jt_host.end(), C, C + 1024);
    }
}

hipError_t jump_table_on_device(size_t entries, const uint64_t **out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_jt_mu);
    JumpTable &t = g_jt[dev];
    if (t.dev_entries < entries) {
        const size_t want = std::max(entries, 2 * t.dev_entries);
        jt_extend_host(want);
        uint64_t *d = nullptr;
        if ((e = hipMalloc(&d, want * 1024 * sizeof(uint64_t))) != hipSuccess) return e;
        if ((e = hipMemcpy(d, g_jt_host.data(), want * 1024 * sizeof(uint64_t), hipMemcpyHostToDevice)) !=
            hipSuccess) {
            (void)hipFree(d);
            return e;
        }
        t.dev = d;  // (the previous, shorter table is left allocated: a launch may still read it)
        t.dev_entries = want;
    }
    *out = t.dev;
    return hipSuccess;
}

}  // namespace

size_t trials_scratch_words(int n, uint64_t n_err, int n_punct, int batch) {
    (void)n;
    (void)n_punct;
    return TrialWs(n_err, batch).words();
}

hipError_t launch_trials(int n, uint64_t n_err, int batch, const uint64_t *seeds, uint64_t seed_add, uint8_t *alice,
                         uint8_t *bob, uint32_t *scratch, int n_punct, uint8_t *punct_alice, uint8_t *punct_bob,
                         hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    if (!scratch || n <= 0 || n_err == 0 || n_err > (uint64_t)n || n_punct < 0) return hipErrorInvalidValue;
    const TrialStream T(n, n_punct);
    const TrialWs W(n_err, batch);
    const size_t nseg = (size_t)T.segments();
    const int ngrp = (batch + 63) / 64;
    if (nseg > 0x7fffffff || ngrp > 65535) return hipErrorInvalidValue;
    const uint64_t *jt = nullptr;
    hipError_t e = jump_table_on_device((size_t)T.units, &jt);
    if (e != hipSuccess) return e;
    // last[] (0 = no writer) and the rejection flags start cleared
    if ((e = hipMemsetAsync(scratch + W.last(), 0, W.k * W.BP * sizeof(uint32_t), stream)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(scratch + W.flag(), 0, W.BP * sizeof(uint32_t), stream)) != hipSuccess) return e;
    const int wide = (n % 16 == 0) && ((reinterpret_cast<uintptr_t>(alice) | reinterpret_cast<uintptr_t>(bob)) & 15) == 0;
    hipLaunchKernelGGL(trials_draw_kernel, dim3((unsigned)nseg, (unsigned)ngrp), dim3(64), 0, stream, n,
                       (uint32_t)n_err, n_punct, batch, seeds, seed_add, jt, wide, alice, bob, punct_alice, punct_bob,
                       scratch);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // QLDPC_TRIAL_SERIAL=1: every trial takes the sequential rerun (the path a
    // rejected draw takes), =2: the one-thread replay of the prefix swaps (the
    // path of kParLds < k <= kPrefixLds); both for the parity tests
    const char *env = qldpc_diag_env("QLDPC_TRIAL_SERIAL");
    const int force_serial = !env ? 0 : std::strcmp(env, "1") == 0 ? 1 : std::strcmp(env, "2") == 0 ? 2 : 0;
    const size_t lds = n_err <= kParLds      ? (3 * (size_t)n_err + 1) * sizeof(uint32_t)
                       : n_err <= kPrefixLds ? 2 * (size_t)n_err * sizeof(uint32_t)
                                             : 0;
    if (lds > 65536 && (e = allow_dynamic_lds(reinterpret_cast<const void *>(trials_finish_kernel), lds)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(trials_finish_kernel, dim3(batch), dim3(256), lds, stream, n, (uint32_t)n_err, n_punct, batch,
                       seeds, seed_add, alice, bob, punct_alice, punct_bob, scratch, force_serial);
    return hipGetLastError();
}

}  // namespace qldpc
