// qkd_ldpc_impl.hpp — the C++ side of the drop-in, generic over the caller's
// types: both the namespace mirror (qkd_ldpc_algorithm.hpp) and the
// replacement translation unit for the reference's src/qkd_ldpc_algorithm.cpp
// (dropin/qkd_ldpc_algorithm.cpp, compiled against the reference's own
// headers and globals) are thin layers over these templates.
//
// Matrix: anything with the reference H_matrix's members
//   std::vector<std::vector<int>> bit_nodes, check_nodes
// (src/array_and_matrix_operations.hpp:60-77).  URBG: any uniform random bit
// generator — XoshiroCpp::Xoshiro256PlusPlus in the reference.
// Errors throw std::runtime_error carrying qldpc_last_error().
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <list>
#include <memory>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "qkd_ldpc_hip.h"

namespace qkd_ldpc_v_amd {
namespace impl {

[[noreturn]] inline void raise(const char *what) {
    throw std::runtime_error(std::string(what) + ": " + qldpc_last_error());
}

// The adjacency of an H as flat arrays: the cache key (compared in full).
struct HKey {
    std::vector<int32_t> rp, ci, cp, ri;
    bool operator==(const HKey &o) const { return rp == o.rp && ci == o.ci && cp == o.cp && ri == o.ri; }
};

template <class Matrix>
HKey key_of(const Matrix &H) {
    HKey k;
    k.rp.assign(H.check_nodes.size() + 1, 0);
    k.cp.assign(H.bit_nodes.size() + 1, 0);
    for (size_t j = 0; j < H.check_nodes.size(); ++j) {
        k.ci.insert(k.ci.end(), H.check_nodes[j].begin(), H.check_nodes[j].end());
        k.rp[j + 1] = (int32_t)k.ci.size();
    }
    for (size_t i = 0; i < H.bit_nodes.size(); ++i) {
        k.ri.insert(k.ri.end(), H.bit_nodes[i].begin(), H.bit_nodes[i].end());
        k.cp[i + 1] = (int32_t)k.ri.size();
    }
    return k;
}

// Device graphs by H CONTENT (the full adjacency is compared on every
// lookup, so an H freed and another allocated at the same address can never
// pick up a stale graph), least recently used first out: at most `capacity`
// graphs stay on the device.  release() / clear() free them explicitly.
class GraphCache {
  public:
    template <class Matrix>
    std::shared_ptr<qldpc_graph> get(const Matrix &H) {
        HKey k = key_of(H);
        std::lock_guard<std::mutex> lk(mu_);
        for (auto it = lru_.begin(); it != lru_.end(); ++it)
            if (it->first == k) {
                lru_.splice(lru_.begin(), lru_, it);
                return lru_.front().second;
            }
        qldpc_graph *g = nullptr;
        if (qldpc_graph_create_checked((int32_t)(k.cp.size() - 1), (int32_t)(k.rp.size() - 1), k.rp.data(),
                                       k.ci.data(), k.cp.data(), k.ri.data(), 0, &g))
            raise("qldpc_graph_create_checked");
        std::shared_ptr<qldpc_graph> sp(g, qldpc_graph_destroy);
        lru_.emplace_front(std::move(k), sp);
        while (lru_.size() > capacity_) lru_.pop_back();  // callers still holding it keep it alive
        return sp;
    }
    // Drop H's graph (device memory is freed once no call uses it).
    template <class Matrix>
    bool release(const Matrix &H) {
        const HKey k = key_of(H);
        std::lock_guard<std::mutex> lk(mu_);
        for (auto it = lru_.begin(); it != lru_.end(); ++it)
            if (it->first == k) {
                lru_.erase(it);
                return true;
            }
        return false;
    }
    void clear() {
        std::lock_guard<std::mutex> lk(mu_);
        lru_.clear();
    }
    void set_capacity(size_t c) {
        std::lock_guard<std::mutex> lk(mu_);
        capacity_ = std::max<size_t>(1, c);
        while (lru_.size() > capacity_) lru_.pop_back();
    }
    size_t size() {
        std::lock_guard<std::mutex> lk(mu_);
        return lru_.size();
    }

  private:
    std::mutex mu_;
    std::list<std::pair<HKey, std::shared_ptr<qldpc_graph>>> lru_;
    size_t capacity_ = 4;
};

inline GraphCache &graph_cache() {
    static GraphCache c;
    return c;
}

// One frame through qldpc_decode_batch: the reference's per-frame decoder
// call (src/qkd_ldpc_algorithm.hpp:28-90).  Returns {iterations_num,
// syndromes_match}; out is resized to n and receives bit_array_out.
template <class Matrix>
std::pair<size_t, bool> decode_one(int32_t alg, const std::vector<double> &llr, const Matrix &H,
                                   const std::vector<int> &syndrome, size_t max_it, double primary, double secondary,
                                   bool thr_enabled, double thr, std::vector<int> &out) {
    const size_t n = H.bit_nodes.size(), m = H.check_nodes.size();
    if (llr.size() < n || syndrome.size() < m) throw std::runtime_error("decode: llr / syndrome shorter than the matrix");
    auto g = graph_cache().get(H);
    std::vector<uint8_t> s(m), bits(n);
    for (size_t j = 0; j < m; ++j) s[j] = (uint8_t)(syndrome[j] & 1);
    qldpc_params p{alg, (int32_t)max_it, thr_enabled ? 1 : 0, 0, thr, primary, secondary};
    uint32_t iters = 0;
    uint8_t ok = 0;
    if (qldpc_decode_batch(g.get(), &p, 1, llr.data(), s.data(), bits.data(), &iters, &ok, nullptr))
        raise("qldpc_decode_batch");
    out.resize(n);
    for (size_t i = 0; i < n; ++i) out[i] = bits[i];
    return {iters, ok != 0};
}

// calculate_syndrome (src/array_and_matrix_operations.cpp:936-950).
template <class Matrix>
void calculate_syndrome(const std::vector<int> &bit_array, const Matrix &H, std::vector<int> &syndrome_out) {
    std::fill(syndrome_out.begin(), syndrome_out.end(), 0);
    for (size_t j = 0; j < H.check_nodes.size(); ++j)
        for (int b : H.check_nodes[j]) syndrome_out[j] ^= bit_array[b];
}

// arrays_equal: compares over array1's length (src/array_and_matrix_operations.cpp:105-118).
inline bool arrays_equal(const std::vector<int> &a, const std::vector<int> &b) {
    for (size_t i = 0; i < a.size(); ++i)
        if (a[i] != b[i]) return false;
    return true;
}

// remove_bits (src/array_and_matrix_operations.cpp:259-287): bits_to_remove ascending.
inline void remove_bits(const std::vector<int> &bits_to_remove, const std::vector<int> &array1,
                        const std::vector<int> &array2, std::vector<int> &array1_out, std::vector<int> &array2_out) {
    const size_t btr = bits_to_remove.size();
    array1_out.resize(array1.size() - btr);
    array2_out.resize(array1.size() - btr);
    size_t r = 0, o = 0;
    for (size_t i = 0; i < array1.size(); ++i) {
        if (r < btr && bits_to_remove[r] == (int)i) {
            ++r;
        } else {
            array1_out[o] = array1[i];
            array2_out[o] = array2[i];
            ++o;
        }
    }
}

// tanh_lin_approx / atanh_lin_approx (src/qkd_ldpc_algorithm.cpp:146-172):
// odd piecewise-linear functions (the device kernels' tanh_lin / atanh_lin).
inline double tanh_lin_approx(double x) {
    const double a = std::fabs(x);
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
inline double atanh_lin_approx(double x) {
    const double a = std::fabs(x);
    double r;
    if (a < 0.7) r = 1.196 * a - 0.0323;
    else if (a < 0.9) r = 2.9187 * a - 1.214;
    else if (a < 0.999) r = 10.8717 * a - 8.3717;
    else r = 2510.9 * a - 2505.9;
    return (x < 0.) ? -r : r;
}

// The hot-path inputs the reference reads from its global CFG.
struct DecodeConfig {
    int32_t algorithm;
    size_t max_iterations;
    bool thr_enabled;
    double thr;
};

struct TrialResult {
    size_t iterations_num;
    bool syndromes_match;
    bool keys_match;
};

// QKD_LDPC (src/qkd_ldpc_algorithm.cpp:1031-1119): Bob's a-priori LLRs
// +-log((1 - q) / q), Alice's syndrome, the configured decoder, keys_match.
// (The privacy-maintenance remove_bits at :1089-1092 only feeds TRACE
// printing and is skipped here.)
template <class Matrix>
TrialResult qkd_ldpc(const Matrix &H, const std::vector<int> &alice, const std::vector<int> &bob, double qber,
                     double primary, double secondary, const DecodeConfig &cfg) {
    const size_t n = H.bit_nodes.size(), m = H.check_nodes.size();
    const double log_p = std::log((1. - qber) / qber);
    std::vector<double> llr(n);
    for (size_t i = 0; i < n; ++i) llr[i] = bob[i] ? -log_p : log_p;
    std::vector<int> synd(m);
    calculate_syndrome(alice, H, synd);
    std::vector<int> out(n);
    const auto r = decode_one(cfg.algorithm, llr, H, synd, cfg.max_iterations, primary, secondary, cfg.thr_enabled,
                              cfg.thr, out);
    return {r.first, r.second, arrays_equal(alice, out)};
}

// QKD_LDPC_RATE_ADAPT (src/qkd_ldpc_algorithm.cpp:1121-1258): the extended
// frame over all n positions — a punctured position takes TWO draws of
// uniform_int_distribution<int>(0, 1) from the caller's generator, Alice's then
// Bob's, in position order (:1148-1157; LLR ALMOST_ZERO = 1e-4), a shortened
// one is 0/0 with LLR DBL_MAX (:1158-1166), any other the next key bit with
// +-log_p (:1167-1172) — then the configured decoder and keys_match against
// the EXTENDED Alice key (:1216).  punctured / shortened: ascending positions.
template <class Matrix, class URBG>
TrialResult qkd_ldpc_rate_adapt(const Matrix &H, const std::vector<int> &alice, const std::vector<int> &bob,
                                double qber, double primary, double secondary, const std::vector<int> &punctured,
                                const std::vector<int> &shortened, URBG &prng, const DecodeConfig &cfg) {
    const size_t n = H.bit_nodes.size(), m = H.check_nodes.size();
    const double log_p = std::log((1. - qber) / qber);
    std::vector<double> llr(n);
    std::vector<int> alice_ext(n), bob_ext(n);
    std::uniform_int_distribution<int> distribution(0, 1);
    size_t p = 0, s = 0, k = 0;
    for (size_t i = 0; i < n; ++i) {
        if (p < punctured.size() && punctured[p] == (int)i) {
            alice_ext[i] = distribution(prng);
            bob_ext[i] = distribution(prng);
            llr[i] = 1e-4;
            ++p;
        } else if (s < shortened.size() && shortened[s] == (int)i) {
            alice_ext[i] = 0;
            bob_ext[i] = 0;
            llr[i] = std::numeric_limits<double>::max();
            ++s;
        } else {
            alice_ext[i] = alice[k];
            bob_ext[i] = bob[k];
            llr[i] = bob[k] ? -log_p : log_p;
            ++k;
        }
    }
    std::vector<int> synd(m);
    calculate_syndrome(alice_ext, H, synd);
    std::vector<int> out(n);
    const auto r = decode_one(cfg.algorithm, llr, H, synd, cfg.max_iterations, primary, secondary, cfg.thr_enabled,
                              cfg.thr, out);
    return {r.first, r.second, arrays_equal(alice_ext, out)};
}

}  // namespace impl
}  // namespace qkd_ldpc_v_amd
