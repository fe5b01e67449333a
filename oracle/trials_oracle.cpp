// trials_oracle.cpp — CPU ORACLE for the reference's trial generator.
//
// TEST INFRASTRUCTURE ONLY (see ldpc_oracle.h).  Restates, per trial,
// run_trial's key generation (ColdCloudd/QKD_LDPC_V src/simulation.cpp:540-551)
// — fill_random_bits + inject_errors (src/array_and_matrix_operations.cpp:
// 889-933) — and the per-trial seeds of the simulation loop
// (src/simulation.cpp:713-719,743: seeds[n] = uniform_int_distribution<size_t>
// over Xoshiro256++(SIMULATION_SEED), trial seed = seeds[n] + curr_sim).
//
// The distributions are the C++ standard library's OWN
// std::uniform_int_distribution and std::shuffle, compiled from this image's
// libstdc++ (GCC 11.4 — the reference's Ubuntu 22.04 toolchain), so their
// draw-consumption and mapping are exact by construction.  The generator is
// Xoshiro256++ restated from its published definition (Blackman & Vigna) with
// Xoshiro-cpp v1.1's seeding (four SplitMix64 outputs), which is absent from
// this image: that part is "parity unpinned" against the upstream header.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

namespace {

struct Xoshiro256pp {  // UniformRandomBitGenerator
    using result_type = uint64_t;
    uint64_t s[4];
    static constexpr uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    explicit Xoshiro256pp(uint64_t seed) {
        uint64_t x = seed;
        for (auto &v : s) {  // SplitMix64
            uint64_t z = (x += 0x9e3779b97f4a7c15ull);
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
            v = z ^ (z >> 31);
        }
    }
    static constexpr result_type min() { return 0; }
    static constexpr result_type max() { return std::numeric_limits<uint64_t>::max(); }
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

extern "C" {

// First `count` outputs of Xoshiro256++(seed) (raw, i.e. the generator's next()).
void qlo_xoshiro(uint64_t seed, int32_t count, uint64_t *out) {
    Xoshiro256pp g(seed);
    for (int32_t i = 0; i < count; ++i) out[i] = g();
}

// seeds[i] as the simulation loop draws them (src/simulation.cpp:713-719).
void qlo_trial_seeds(uint64_t simulation_seed, int32_t count, uint64_t *seeds) {
    Xoshiro256pp g(simulation_seed);
    std::uniform_int_distribution<size_t> d(0, std::numeric_limits<size_t>::max());
    for (int32_t i = 0; i < count; ++i) seeds[i] = d(g);
}

// One trial's keys (src/simulation.cpp:548-551): alice = fill_random_bits,
// bob = inject_errors(alice, qber).  Returns the accurate QBER.
double qlo_trial(int32_t n, double qber, uint64_t seed, uint8_t *alice, uint8_t *bob) {
    Xoshiro256pp g(seed);
    std::vector<int> a(n), b;
    std::uniform_int_distribution<int> bit(0, 1);
    for (int32_t i = 0; i < n; ++i) a[i] = bit(g);
    const size_t ne = static_cast<size_t>(static_cast<double>(n) * qber);
    b = a;
    if (ne > 0) {
        std::vector<size_t> pos(n);
        for (int32_t i = 0; i < n; ++i) pos[i] = (size_t)i;
        std::shuffle(pos.begin(), pos.end(), g);
        for (size_t i = 0; i < ne; ++i) b[pos[i]] ^= 1;
    }
    for (int32_t i = 0; i < n; ++i) {
        alice[i] = (uint8_t)a[i];
        bob[i] = (uint8_t)b[i];
    }
    return static_cast<double>(ne) / static_cast<double>(n);
}

}  // extern "C"

// ---- rate adaptation (src/array_and_matrix_operations.cpp:1131-1223;
//      src/qkd_ldpc_algorithm.cpp:1121-1180) ---------------------------------
extern "C" {

// adapt_code_rate over a generator whose 4-word state is advanced in place.
// Returns 0 and counts (0/0 for the reference's skipped combinations).
int qlo_adapt_code_rate(int32_t n, int32_t m, double qber, double delta, double efficiency, int32_t untainted_on,
                        const int32_t *untainted, int32_t n_untainted, uint64_t *state, int32_t *punct,
                        int32_t *n_punct, int32_t *shortened, int32_t *n_short) {
    Xoshiro256pp g(0);
    std::memcpy(g.s, state, sizeof g.s);
    *n_punct = *n_short = 0;
    const double h_b = -qber * std::log2(qber) - (1. - qber) * std::log2(1. - qber);
    const double optimal_R = 1. - efficiency * h_b;
    const double original_R = 1. - static_cast<double>(m) / static_cast<double>(n);
    const int ns = static_cast<int>(std::ceil((original_R - optimal_R * (1. - delta)) * static_cast<double>(n)));
    const int np = static_cast<int>(delta * static_cast<double>(n) - static_cast<double>(ns));
    if (ns <= 0 || np <= 0) return 0;
    std::vector<int> p, pos(n);
    if (untainted_on) {
        if (np > n_untainted) return 0;
        p.assign(untainted, untainted + np);
    } else {
        for (int i = 0; i < n; ++i) pos[i] = i;
        std::shuffle(pos.begin(), pos.end(), g);
        p.assign(pos.begin(), pos.begin() + np);
    }
    std::sort(p.begin(), p.end());
    for (int i = 0; i < n; ++i) pos[i] = i;
    std::vector<int> rem(n - np);
    std::set_difference(pos.begin(), pos.end(), p.begin(), p.end(), rem.begin());
    std::shuffle(rem.begin(), rem.end(), g);
    std::vector<int> s(rem.begin(), rem.begin() + ns);
    std::sort(s.begin(), s.end());
    std::memcpy(state, g.s, sizeof g.s);
    std::copy(p.begin(), p.end(), punct);
    std::copy(s.begin(), s.end(), shortened);
    *n_punct = np;
    *n_short = ns;
    return 0;
}

// A rate-adapted trial: run_trial's keys, then QKD_LDPC_RATE_ADAPT's extended
// frame.  Outputs alice_ext[n], llr[n]; returns the accurate QBER.
double qlo_trial_rate_adapt(int32_t n, double qber, uint64_t seed, int32_t n_punct, const int32_t *punct,
                            int32_t n_short, const int32_t *shortened, uint8_t *alice_ext, double *llr) {
    Xoshiro256pp g(seed);
    std::vector<int> a(n), b;
    std::uniform_int_distribution<int> bit(0, 1);
    for (int32_t i = 0; i < n; ++i) a[i] = bit(g);
    const size_t ne = static_cast<size_t>(static_cast<double>(n) * qber);
    b = a;
    std::vector<size_t> pos(n);
    for (int32_t i = 0; i < n; ++i) pos[i] = (size_t)i;
    std::shuffle(pos.begin(), pos.end(), g);
    for (size_t i = 0; i < ne; ++i) b[pos[i]] ^= 1;
    const double q = static_cast<double>(ne) / static_cast<double>(n);
    const double log_p = std::log((1. - q) / q);
    int p = 0, s = 0, k = 0;
    for (int i = 0; i < n; ++i) {
        if (p < n_punct && punct[p] == i) {
            alice_ext[i] = (uint8_t)bit(g);
            (void)bit(g);  // Bob's punctured bit
            llr[i] = 1e-4;
            ++p;
        } else if (s < n_short && shortened[s] == i) {
            alice_ext[i] = 0;
            llr[i] = std::numeric_limits<double>::max();
            ++s;
        } else {
            alice_ext[i] = (uint8_t)a[k];
            llr[i] = b[k] ? -log_p : log_p;
            ++k;
        }
    }
    return q;
}

}  // extern "C"
