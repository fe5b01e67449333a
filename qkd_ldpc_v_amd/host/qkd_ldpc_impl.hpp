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
#include <condition_variable>
#include <cstdlib>
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

// The adjacency of an H as flat CSR (check_nodes) + CSC (bit_nodes) arrays.
struct HFlat {
    std::vector<int32_t> rp, ci, cp, ri;
};

template <class Matrix>
HFlat flatten(const Matrix &H) {
    HFlat k;
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

// Content fingerprint of an H: n, m, every list's length and every entry,
// in list order, mixed four lanes at a time (64-bit multiply-xorshift; no
// allocation).  Read without any lock, so concurrent callers hash in parallel.
struct HKey {
    uint64_t h = 0;
    size_t n = 0, m = 0, nnz = 0;
    bool operator==(const HKey &o) const { return h == o.h && n == o.n && m == o.m && nnz == o.nnz; }
};

inline uint64_t mix64(uint64_t x) {
    x ^= x >> 31;
    x *= 0x7fb5d329728ea185ull;
    x ^= x >> 27;
    x *= 0x81dadef4bc2dd44dull;
    return x ^ (x >> 33);
}

template <class Lists>
void hash_lists(const Lists &L, uint64_t acc[4], size_t &nnz) {
    for (const auto &v : L) {
        acc[0] = (acc[0] ^ (uint64_t)v.size()) * 0x9e3779b97f4a7c15ull;
        const int *d = v.data();
        const size_t k = v.size();
        size_t i = 0;
        for (; i + 4 <= k; i += 4)
            for (int l = 0; l < 4; ++l) acc[l] = (acc[l] ^ (uint32_t)d[i + l]) * 0xff51afd7ed558ccdull + (uint64_t)l;
        for (; i < k; ++i) acc[i & 3] = (acc[i & 3] ^ (uint32_t)d[i]) * 0xc4ceb9fe1a85ec53ull;
        nnz += k;
    }
}

template <class Matrix>
HKey key_of(const Matrix &H) {
    uint64_t acc[4] = {0x243f6a8885a308d3ull, 0x13198a2e03707344ull, 0xa4093822299f31d0ull, 0x082efa98ec4e6c89ull};
    size_t nnz_c = 0, nnz_b = 0;
    hash_lists(H.check_nodes, acc, nnz_c);
    const uint64_t sep = mix64(acc[0] ^ mix64(acc[1]) ^ mix64(acc[2] + 1) ^ mix64(acc[3] + 2));
    acc[0] ^= sep;
    hash_lists(H.bit_nodes, acc, nnz_b);
    HKey k;
    k.h = mix64(acc[0] ^ mix64(acc[1] ^ mix64(acc[2] ^ mix64(acc[3] ^ sep))));
    k.n = H.bit_nodes.size();
    k.m = H.check_nodes.size();
    k.nnz = nnz_c | (nnz_b << 32);
    return k;
}

// The O(1) part of the cache lookup: the H object's address, its two outer
// buffers and sizes, and a fingerprint of 64 evenly spaced check rows and 64
// bit columns (their buffer addresses, lengths and entries).  A hit on it is
// trusted; anything else — another object, a reloaded or reassigned H, a
// rewritten sampled list — falls back to the full content fingerprint.
struct HFastKey {
    const void *obj = nullptr, *rows = nullptr, *cols = nullptr;
    size_t n = 0, m = 0;
    uint64_t sample = 0;
    bool operator==(const HFastKey &o) const {
        return obj == o.obj && rows == o.rows && cols == o.cols && n == o.n && m == o.m && sample == o.sample;
    }
};

template <class Lists>
uint64_t sample_lists(const Lists &L, uint64_t acc) {
    const size_t cnt = L.size(), step = cnt > 64 ? cnt / 64 : 1;
    for (size_t j = 0; j < cnt; j += step) {
        const auto &v = L[j];
        acc = mix64(acc ^ (uint64_t)(uintptr_t)v.data() ^ ((uint64_t)v.size() << 48) ^ j);
        for (int x : v) acc = (acc ^ (uint32_t)x) * 0x9e3779b97f4a7c15ull;
    }
    return acc;
}

template <class Matrix>
HFastKey fast_key_of(const Matrix &H) {
    HFastKey k;
    k.obj = &H;
    k.rows = H.check_nodes.data();
    k.cols = H.bit_nodes.data();
    k.n = H.bit_nodes.size();
    k.m = H.check_nodes.size();
    k.sample = mix64(sample_lists(H.bit_nodes, sample_lists(H.check_nodes, 0x6a09e667f3bcc908ull)));
    return k;
}

// The devices the drop-in's graphs live on: QKD_LDPC_HIP_DEVICES (a comma
// list of HIP device ids; a device may repeat: logical shards of one GPU), or
// every GPU of the node.  Read once.
inline const std::vector<int32_t> &drop_in_devices() {
    static const std::vector<int32_t> devs = [] {
        std::vector<int32_t> d;
        if (const char *e = std::getenv("QKD_LDPC_HIP_DEVICES")) {
            std::string s(e);
            size_t pos = 0;
            while (pos < s.size()) {
                size_t q = s.find(',', pos);
                if (q == std::string::npos) q = s.size();
                if (q > pos) d.push_back((int32_t)std::stoi(s.substr(pos, q - pos)));
                pos = q + 1;
            }
        }
        if (d.empty()) {
            int32_t c = 0;
            if (qldpc_device_count(&c) || c <= 0) raise("qldpc_device_count");
            for (int32_t i = 0; i < c; ++i) d.push_back(i);
        }
        return d;
    }();
    return devs;
}

// Group commit of the per-frame decoder calls the reference's thread pool makes
// concurrently (src/simulation.cpp:740-745: THREADS_NUMBER threads, one
// run_trial each): a caller that finds no batch in flight becomes the leader,
// takes every queued frame with the same decoder parameters, decodes them as
// ONE qldpc_decode_batch (sharded over the graph's devices), hands each caller
// its own result, and the next leader takes whatever queued meanwhile.  A lone
// caller decodes its frame alone; results never depend on the grouping (every
// frame is decoded independently).
class Coalescer {
  public:
    struct Req {
        qldpc_params p{};
        const double *llr = nullptr;
        const uint8_t *synd = nullptr;
        uint8_t *bits = nullptr;
        uint32_t iters = 0;
        uint8_t ok = 0;
        int rc = 0;
        std::string err;
        bool done = false;
    };

    void decode(qldpc_graph *g, size_t n, size_t m, Req &r) {
        std::unique_lock<std::mutex> lk(mu_);
        q_.push_back(&r);
        while (!r.done) {
            if (busy_) {
                cv_.wait(lk);
                continue;
            }
            busy_ = true;
            std::vector<Req *> b;
            const qldpc_params p0 = q_.front()->p;
            for (auto it = q_.begin(); it != q_.end();) {
                if (same(p0, (*it)->p)) {
                    b.push_back(*it);
                    it = q_.erase(it);
                } else {
                    ++it;
                }
            }
            lk.unlock();
            try {
                run(g, n, m, p0, b);
            } catch (const std::exception &e) {  // (e.g. bad_alloc staging the batch)
                for (Req *x : b) {
                    x->rc = -1;
                    x->err = e.what();
                }
            } catch (...) {
                for (Req *x : b) {
                    x->rc = -1;
                    x->err = "unknown exception";
                }
            }
            lk.lock();
            // every caller of the batch is released and the next leader may
            // start, whatever run() did
            for (Req *x : b) x->done = true;
            busy_ = false;
            cv_.notify_all();
        }
    }

    // frames decoded / batches launched (diagnostics)
    size_t frames() const { return frames_; }
    size_t batches() const { return batches_; }

  private:
    static bool same(const qldpc_params &a, const qldpc_params &b) {
        return a.algorithm == b.algorithm && a.max_iterations == b.max_iterations && a.thr_enabled == b.thr_enabled &&
               std::memcmp(&a.thr, &b.thr, sizeof(double)) == 0 &&
               std::memcmp(&a.primary, &b.primary, sizeof(double)) == 0 &&
               std::memcmp(&a.secondary, &b.secondary, sizeof(double)) == 0;
    }
    void run(qldpc_graph *g, size_t n, size_t m, const qldpc_params &p, std::vector<Req *> &b) {
        const size_t B = b.size();
        llr_.resize(B * n);
        syn_.resize(B * m);
        bits_.resize(B * n);
        it_.resize(B);
        ok_.resize(B);
        for (size_t f = 0; f < B; ++f) {
            std::memcpy(llr_.data() + f * n, b[f]->llr, n * sizeof(double));
            std::memcpy(syn_.data() + f * m, b[f]->synd, m);
        }
        const int rc = qldpc_decode_batch(g, &p, (int32_t)B, llr_.data(), syn_.data(), bits_.data(), it_.data(),
                                          ok_.data(), nullptr);
        const std::string err = rc ? std::string(qldpc_last_error()) : std::string();
        for (size_t f = 0; f < B; ++f) {
            Req &r = *b[f];
            r.rc = rc;
            if (rc) {
                r.err = err;
                continue;
            }
            std::memcpy(r.bits, bits_.data() + f * n, n);
            r.iters = it_[f];
            r.ok = ok_[f];
        }
        frames_ += B;
        ++batches_;
    }

    std::mutex mu_;
    std::condition_variable cv_;
    std::list<Req *> q_;
    bool busy_ = false;
    // the leader's staging buffers (one leader at a time)
    std::vector<double> llr_;
    std::vector<uint8_t> syn_, bits_, ok_;
    std::vector<uint32_t> it_;
    size_t frames_ = 0, batches_ = 0;
};

// A cached device graph and its per-frame call coalescer.
struct GraphEntry {
    std::shared_ptr<qldpc_graph> g;
    Coalescer co;
};

// Device graphs by H CONTENT, least recently used first out: at most
// `capacity` graphs stay on the devices.  A call first looks up its O(1)
// fast key (HFastKey: the same object, buffers and sampled lists as a call
// already resolved); on a miss it takes the fingerprint of every list
// (HKey, one pass over the adjacency, computed without any lock), so an H
// freed and another allocated at the same address, or an H reloaded in place
// (the reference's config-after-config loop), never picks up a stale graph.
// An in-place edit that leaves all 128 sampled lists unchanged is seen by the
// fast key only at an entry's next full check (every kVerifyEvery-th hit):
// call release() after one to drop the graph at once.  DESIGN.md §2 has the
// costs.
class GraphCache {
  public:
    template <class Matrix>
    std::shared_ptr<GraphEntry> get(const Matrix &H) {
        const HFastKey fk = fast_key_of(H);
        {
            std::shared_ptr<GraphEntry> hit;
            HKey hk;
            {
                std::lock_guard<std::mutex> lk(mu_);
                for (auto it = lru_.begin(); it != lru_.end(); ++it)
                    if (it->fast == fk) {
                        lru_.splice(lru_.begin(), lru_, it);
                        // every kVerifyEvery-th hit of an entry re-checks the whole
                        // content, so an in-place edit the sampled lists miss is
                        // caught within that many calls (release() at once)
                        if (++it->hits % kVerifyEvery != 0) return lru_.front().e;
                        hit = it->e;
                        hk = it->key;
                        break;
                    }
            }
            if (hit && key_of(H) == hk) return hit;
        }
        const HKey k = key_of(H);
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (auto it = lru_.begin(); it != lru_.end(); ++it)
                if (it->key == k) {
                    it->fast = fk;  // (the newest object holding this content)
                    lru_.splice(lru_.begin(), lru_, it);
                    return lru_.front().e;
                }
        }
        // a miss: build the graph outside the lock (first-come wins a race)
        const HFlat f = flatten(H);
        const auto &devs = drop_in_devices();
        qldpc_graph *g = nullptr;
        if (qldpc_graph_create_checked_on((int32_t)(f.cp.size() - 1), (int32_t)(f.rp.size() - 1), f.rp.data(),
                                          f.ci.data(), f.cp.data(), f.ri.data(), devs.data(), (int32_t)devs.size(),
                                          &g))
            raise("qldpc_graph_create_checked_on");
        auto e = std::make_shared<GraphEntry>();
        e->g = std::shared_ptr<qldpc_graph>(g, qldpc_graph_destroy);
        std::lock_guard<std::mutex> lk(mu_);
        for (auto it = lru_.begin(); it != lru_.end(); ++it)
            if (it->key == k) {
                it->fast = fk;
                lru_.splice(lru_.begin(), lru_, it);
                return lru_.front().e;
            }
        lru_.push_front(Slot{k, fk, e, 0});
        while (lru_.size() > capacity_) lru_.pop_back();  // callers still holding it keep it alive
        return e;
    }
    // Drop H's graph (device memory is freed once no call uses it).
    template <class Matrix>
    bool release(const Matrix &H) {
        const HKey k = key_of(H);
        const HFastKey fk = fast_key_of(H);
        std::lock_guard<std::mutex> lk(mu_);
        bool hit = false;
        for (auto it = lru_.begin(); it != lru_.end();) {
            if (it->key == k || it->fast == fk) {
                it = lru_.erase(it);
                hit = true;
            } else {
                ++it;
            }
        }
        return hit;
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
    struct Slot {
        HKey key;
        HFastKey fast;
        std::shared_ptr<GraphEntry> e;
        uint64_t hits = 0;
    };
    static constexpr uint64_t kVerifyEvery = 32;
    std::mutex mu_;
    std::list<Slot> lru_;
    size_t capacity_ = 4;
};

inline GraphCache &graph_cache() {
    static GraphCache c;
    return c;
}

// One frame through the coalesced qldpc_decode_batch: the reference's
// per-frame decoder call (src/qkd_ldpc_algorithm.hpp:28-90).  Returns
// {iterations_num, syndromes_match}; out is resized to n and receives
// bit_array_out.  The syndrome must hold 0 / 1 (what calculate_syndrome
// produces, src/array_and_matrix_operations.cpp:936-950): the kernels take
// bits, while the reference's decoders would treat any other value as a sign
// flip (:57) that can never match (:101) — that input is refused.
template <class Matrix>
std::pair<size_t, bool> decode_one(int32_t alg, const std::vector<double> &llr, const Matrix &H,
                                   const std::vector<int> &syndrome, size_t max_it, double primary, double secondary,
                                   bool thr_enabled, double thr, std::vector<int> &out) {
    const size_t n = H.bit_nodes.size(), m = H.check_nodes.size();
    if (llr.size() < n || syndrome.size() < m) throw std::runtime_error("decode: llr / syndrome shorter than the matrix");
    std::vector<uint8_t> s(m), bits(n);
    for (size_t j = 0; j < m; ++j) {
        if (syndrome[j] != 0 && syndrome[j] != 1)
            throw std::runtime_error("decode: syndrome[" + std::to_string(j) + "] = " + std::to_string(syndrome[j]) +
                                     " is not a bit (0 or 1)");
        s[j] = (uint8_t)syndrome[j];
    }
    auto e = graph_cache().get(H);
    Coalescer::Req r;
    r.p = qldpc_params{alg, (int32_t)max_it, thr_enabled ? 1 : 0, 0, thr, primary, secondary};
    r.llr = llr.data();
    r.synd = s.data();
    r.bits = bits.data();
    e->co.decode(e->g.get(), n, m, r);
    if (r.rc) throw std::runtime_error("qldpc_decode_batch: " + r.err);
    out.resize(n);
    for (size_t i = 0; i < n; ++i) out[i] = bits[i];
    return {r.iters, r.ok != 0};
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

// One trial of the batch seam: the fields run_trial fills in trial_result
// (src/simulation.hpp:36-41; LDPC_result, src/qkd_ldpc_algorithm.hpp:16-26).
struct BatchTrial {
    size_t iterations_num;
    bool syndromes_match;
    bool keys_match;
    double runtime_us;  // trial_result::runtime (qldpc_run_trials: share of the chunk window)
};

// One combination's trials on the devices (qldpc_run_trials_submit): holds
// the device graph, the rate plan and the result arrays until wait() (which
// the destructor also does, so a job never leaves chunks behind).
class TrialsJob {
  public:
    TrialsJob(std::shared_ptr<GraphEntry> e, qldpc_rate_plan *plan, size_t count)
        : e_(std::move(e)), plan_(plan, qldpc_rate_plan_destroy), it_(count), ok_(count), km_(count), rt_(count) {}
    TrialsJob(const TrialsJob &) = delete;
    TrialsJob &operator=(const TrialsJob &) = delete;
    ~TrialsJob() {
        if (h_) (void)qldpc_run_trials_wait(h_);
    }
    // Per trial {iterations_num, syndromes_match, keys_match, runtime_us}.
    std::vector<BatchTrial> wait() {
        qldpc_trials_job *h = h_;
        h_ = nullptr;
        if (h && qldpc_run_trials_wait(h)) throw std::runtime_error(qldpc_last_error());
        std::vector<BatchTrial> out(it_.size());
        for (size_t t = 0; t < out.size(); ++t) out[t] = {it_[t], ok_[t] != 0, km_[t] != 0, rt_[t]};
        return out;
    }
    double accurate_qber() const { return q_; }

  private:
    template <class Matrix>
    friend std::unique_ptr<TrialsJob> submit_trials(const Matrix &, double, const std::vector<size_t> &, size_t,
                                                    double, double, const DecodeConfig &, const std::vector<int> *,
                                                    const std::vector<int> *);
    std::shared_ptr<GraphEntry> e_;
    std::unique_ptr<qldpc_rate_plan, void (*)(qldpc_rate_plan *)> plan_;
    std::vector<uint32_t> it_;
    std::vector<uint8_t> ok_, km_;
    std::vector<double> rt_;
    double q_ = 0.;
    qldpc_trials_job *h_ = nullptr;
};

// The batch seam of the simulation loop: run_trial for every seed of one
// combination (QKD_LDPC_batch_simulation's pool.detach_loop over run_trial,
// src/simulation.cpp:721-746), submitted as one qldpc_run_trials_submit —
// trial t uses the seed seeds[t] + seed_add (the loop's `seeds[n] +
// curr_sim`, :743); the trials are generated, decoded and compared on the
// drop-in's devices, sharded over them, while the caller goes on (e.g. to
// submit the next combination).  punctured / shortened (ascending, both or
// neither): CFG.ENABLE_CODE_RATE_ADAPTATION's QKD_LDPC_RATE_ADAPT, else
// QKD_LDPC.  Throws run_trial's errors (e.g. "Key size ... is too small for
// QBER.").
template <class Matrix>
std::unique_ptr<TrialsJob> submit_trials(const Matrix &H, double qber, const std::vector<size_t> &seeds,
                                         size_t seed_add, double primary, double secondary, const DecodeConfig &cfg,
                                         const std::vector<int> *punctured, const std::vector<int> *shortened) {
    auto e = graph_cache().get(H);
    qldpc_rate_plan *plan = nullptr;
    if (punctured && shortened &&
        qldpc_rate_plan_create(e->g.get(), (int32_t)punctured->size(), punctured->data(), (int32_t)shortened->size(),
                               shortened->data(), &plan))
        raise("qldpc_rate_plan_create");
    std::unique_ptr<TrialsJob> job(new TrialsJob(e, plan, seeds.size()));
    std::vector<uint64_t> sd(seeds.begin(), seeds.end());
    const qldpc_params p{cfg.algorithm, (int32_t)cfg.max_iterations, cfg.thr_enabled ? 1 : 0, 0, cfg.thr, primary,
                         secondary};
    if (qldpc_run_trials_submit(e->g.get(), plan, &p, qber, (int32_t)sd.size(), sd.data(), (uint64_t)seed_add,
                                job->it_.data(), job->ok_.data(), job->km_.data(), job->rt_.data(), &job->q_,
                                &job->h_))
        throw std::runtime_error(qldpc_last_error());
    return job;
}

// run_trials: one combination, submitted and collected (accurate_qber
// nullable: every trial's trial_result::accurate_QBER).
template <class Matrix>
std::vector<BatchTrial> run_trials(const Matrix &H, double qber, const std::vector<size_t> &seeds, size_t seed_add,
                                   double primary, double secondary, const DecodeConfig &cfg,
                                   const std::vector<int> *punctured, const std::vector<int> *shortened,
                                   double *accurate_qber) {
    auto job = submit_trials(H, qber, seeds, seed_add, primary, secondary, cfg, punctured, shortened);
    auto out = job->wait();
    if (accurate_qber) *accurate_qber = job->accurate_qber();
    return out;
}

}  // namespace impl
}  // namespace qkd_ldpc_v_amd
