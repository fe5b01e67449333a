// qkd_ldpc_algorithm.hpp — C++ mirror of the reference's decode interface,
// backed by libqkdldpc_hip.so (include/qkd_ldpc_hip.h).
//
// Same names, argument meaning and error behaviour as ColdCloudd/QKD_LDPC_V:
//   H_matrix                  src/array_and_matrix_operations.hpp:60-77
//   read_sparse_*             src/array_and_matrix_operations.cpp:291-886
//   decoding_result, LDPC_result, the six decoders, QKD_LDPC
//                             src/qkd_ldpc_algorithm.hpp:16-99
//   calculate_syndrome, arrays_equal, remove_bits
//                             src/array_and_matrix_operations.cpp:105-118,259-287,936-950
//   config_data / CFG (the subset the hot path reads)   src/config.hpp:103-198
// A caller of the reference switches by including this header instead: every
// decoder call runs on the GPU.  decode_batch() is the batched entry a driver
// uses in place of the per-trial thread pool (src/simulation.cpp:740-746).
// Errors are std::runtime_error carrying qldpc_last_error().
#pragma once

#include <cmath>
#include <cstdint>
#include <filesystem>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "qkd_ldpc_hip.h"

namespace qkd_ldpc_v_amd {

inline constexpr size_t DEC_SPA = 0, DEC_SPA_APPROX = 1, DEC_NMSA = 2, DEC_OMSA = 3, DEC_ANMSA = 4, DEC_AOMSA = 5;
inline constexpr size_t MAT_SPARSE_UNCOMPRESSED = 0, MAT_SPARSE_ALIST = 1, MAT_SPARSE_1 = 2, MAT_SPARSE_2 = 3;
inline const double ALMOST_ZERO = 1e-4;  // src/qkd_ldpc_algorithm.hpp:13

// The configuration fields the decode path reads (src/config.hpp:103-196).
struct config_data {
    size_t DECODING_ALGORITHM{};
    size_t DECODING_ALG_MAX_ITERATIONS{};
    bool ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD{};
    double DECODING_ALG_MSG_LLR_THRESHOLD{};
    bool ENABLE_PRIVACY_MAINTENANCE{};
};
inline config_data CFG;

struct H_matrix {
    std::vector<std::vector<int>> bit_nodes{};
    std::vector<std::vector<int>> check_nodes{};
    std::vector<int> punctured_bits_untainted{};
    bool is_regular{};
};

struct decoding_scaling_factors {
    double primary{};
    double secondary{};
};

struct H_matrix_params {
    double delta{}, efficiency{}, punctured_fraction{}, shortened_fraction{}, adapted_code_rate{};
    std::vector<int> punctured_bits{}, shortened_bits{}, bits_to_remove{};
};

struct decoding_result {
    size_t iterations_num{};
    bool syndromes_match{};
};

struct LDPC_result {
    decoding_result decoding_res{};
    bool keys_match{};
};

namespace detail {

[[noreturn]] inline void raise(const char *what) {
    throw std::runtime_error(std::string(what) + ": " + qldpc_last_error());
}

inline H_matrix load(const std::filesystem::path &p, int32_t format) {
    int32_t n = 0, m = 0, nnz = 0, reg = 0;
    if (qldpc_load_matrix(p.c_str(), format, &n, &m, &nnz, nullptr, nullptr, nullptr, nullptr, &reg))
        throw std::runtime_error(qldpc_last_error());
    std::vector<int32_t> rp(m + 1), ci(nnz), cp(n + 1), ri(nnz);
    if (qldpc_load_matrix(p.c_str(), format, &n, &m, &nnz, rp.data(), ci.data(), cp.data(), ri.data(), &reg))
        throw std::runtime_error(qldpc_last_error());
    H_matrix H;
    H.is_regular = reg != 0;
    H.check_nodes.resize(m);
    for (int j = 0; j < m; ++j) H.check_nodes[j].assign(ci.begin() + rp[j], ci.begin() + rp[j + 1]);
    H.bit_nodes.resize(n);
    for (int i = 0; i < n; ++i) H.bit_nodes[i].assign(ri.begin() + cp[i], ri.begin() + cp[i + 1]);
    return H;
}

// One device graph per distinct H (keyed by address + shape; the reference
// passes the same const H_matrix& to every trial).
struct GraphCache {
    std::mutex mu;
    std::map<const H_matrix *, std::pair<size_t, std::shared_ptr<qldpc_graph>>> graphs;

    std::shared_ptr<qldpc_graph> get(const H_matrix &H) {
        size_t nnz = 0;
        for (const auto &r : H.check_nodes) nnz += r.size();
        const size_t key = H.bit_nodes.size() * 1000003u ^ H.check_nodes.size() * 7919u ^ nnz;
        std::lock_guard<std::mutex> lk(mu);
        auto it = graphs.find(&H);
        if (it != graphs.end() && it->second.first == key) return it->second.second;
        std::vector<int32_t> rp(H.check_nodes.size() + 1, 0), ci, cp(H.bit_nodes.size() + 1, 0), ri;
        for (size_t j = 0; j < H.check_nodes.size(); ++j) {
            ci.insert(ci.end(), H.check_nodes[j].begin(), H.check_nodes[j].end());
            rp[j + 1] = (int32_t)ci.size();
        }
        for (size_t i = 0; i < H.bit_nodes.size(); ++i) {
            ri.insert(ri.end(), H.bit_nodes[i].begin(), H.bit_nodes[i].end());
            cp[i + 1] = (int32_t)ri.size();
        }
        qldpc_graph *g = nullptr;
        if (qldpc_graph_create_checked((int32_t)H.bit_nodes.size(), (int32_t)H.check_nodes.size(), rp.data(),
                                       ci.data(), cp.data(), ri.data(), 0, &g))
            raise("qldpc_graph_create_checked");
        std::shared_ptr<qldpc_graph> sp(g, qldpc_graph_destroy);
        graphs[&H] = {key, sp};
        return sp;
    }
};
inline GraphCache graph_cache;

inline decoding_result decode_one(int32_t alg, const std::vector<double> &llr, const H_matrix &H,
                                  const std::vector<int> &syndrome, size_t max_it, double primary, double secondary,
                                  double thr, std::vector<int> &out) {
    auto g = graph_cache.get(H);
    const size_t n = H.bit_nodes.size(), m = H.check_nodes.size();
    std::vector<uint8_t> s(m), bits(n);
    for (size_t j = 0; j < m; ++j) s[j] = (uint8_t)(syndrome[j] & 1);
    qldpc_params p{alg, (int32_t)max_it, CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD ? 1 : 0, 0, thr, primary, secondary};
    uint32_t iters = 0;
    uint8_t ok = 0;
    if (qldpc_decode_batch(g.get(), &p, 1, llr.data(), s.data(), bits.data(), &iters, &ok, nullptr))
        raise("qldpc_decode_batch");
    out.resize(n);
    for (size_t i = 0; i < n; ++i) out[i] = bits[i];
    return {iters, ok != 0};
}

}  // namespace detail

// ---- loaders ---------------------------------------------------------------
inline H_matrix read_sparse_uncompressed_matrix(const std::filesystem::path &p) { return detail::load(p, 0); }
inline H_matrix read_sparse_matrix_alist(const std::filesystem::path &p) { return detail::load(p, 1); }
inline H_matrix read_sparse_matrix_1(const std::filesystem::path &p) { return detail::load(p, 2); }
inline H_matrix read_sparse_matrix_2(const std::filesystem::path &p) { return detail::load(p, 3); }

// ---- array helpers ---------------------------------------------------------
inline void calculate_syndrome(const std::vector<int> &bit_array, const H_matrix &matrix,
                               std::vector<int> &syndrome_out) {
    std::fill(syndrome_out.begin(), syndrome_out.end(), 0);
    for (size_t i = 0; i < matrix.check_nodes.size(); ++i)
        for (int b : matrix.check_nodes[i]) syndrome_out[i] ^= bit_array[b];
}

inline bool arrays_equal(const std::vector<int> &a, const std::vector<int> &b) {
    for (size_t i = 0; i < a.size(); ++i)
        if (a[i] != b[i]) return false;
    return true;
}

inline void remove_bits(const std::vector<int> &bits_to_remove, const std::vector<int> &array1,
                        const std::vector<int> &array2, std::vector<int> &array1_out, std::vector<int> &array2_out) {
    const size_t btr = bits_to_remove.size();
    array1_out.resize(array1.size() - btr);
    array2_out.resize(array1.size() - btr);
    size_t n = 0, m = 0;
    for (size_t i = 0; i < array1.size(); ++i) {
        if (n < btr && bits_to_remove[n] == (int)i) {
            ++n;
        } else {
            array1_out[m] = array1[i];
            array2_out[m] = array2[i];
            ++m;
        }
    }
}

// ---- the six decoders (src/qkd_ldpc_algorithm.hpp:28-90) -------------------
inline decoding_result sum_product_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                            const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                            const double &msg_threshold, std::vector<int> &bit_array_out) {
    return detail::decode_one(QLDPC_SPA, bit_array_llr, matrix, syndrome, max_num_iterations, 0, 0, msg_threshold,
                              bit_array_out);
}
inline decoding_result sum_product_linear_approx_decoding(const std::vector<double> &bit_array_llr,
                                                          const H_matrix &matrix, const std::vector<int> &syndrome,
                                                          const size_t &max_num_iterations,
                                                          const double &msg_threshold,
                                                          std::vector<int> &bit_array_out) {
    return detail::decode_one(QLDPC_SPA_LIN, bit_array_llr, matrix, syndrome, max_num_iterations, 0, 0,
                              msg_threshold, bit_array_out);
}
inline decoding_result min_sum_normalized_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                                   const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                                   const double &alpha, const double &msg_threshold,
                                                   std::vector<int> &bit_array_out) {
    return detail::decode_one(QLDPC_NMSA, bit_array_llr, matrix, syndrome, max_num_iterations, alpha, 0,
                              msg_threshold, bit_array_out);
}
inline decoding_result min_sum_offset_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                               const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                               const double &beta, const double &msg_threshold,
                                               std::vector<int> &bit_array_out) {
    return detail::decode_one(QLDPC_OMSA, bit_array_llr, matrix, syndrome, max_num_iterations, beta, 0,
                              msg_threshold, bit_array_out);
}
inline decoding_result adaptive_min_sum_normalized_decoding(const std::vector<double> &bit_array_llr,
                                                            const H_matrix &matrix, const std::vector<int> &syndrome,
                                                            const size_t &max_num_iterations, const double &alpha,
                                                            const double &nu, const double &msg_threshold,
                                                            std::vector<int> &bit_array_out) {
    return detail::decode_one(QLDPC_ANMSA, bit_array_llr, matrix, syndrome, max_num_iterations, alpha, nu,
                              msg_threshold, bit_array_out);
}
inline decoding_result adaptive_min_sum_offset_decoding(const std::vector<double> &bit_array_llr,
                                                        const H_matrix &matrix, const std::vector<int> &syndrome,
                                                        const size_t &max_num_iterations, const double &beta,
                                                        const double &sigma, const double &msg_threshold,
                                                        std::vector<int> &bit_array_out) {
    return detail::decode_one(QLDPC_AOMSA, bit_array_llr, matrix, syndrome, max_num_iterations, beta, sigma,
                              msg_threshold, bit_array_out);
}

// ---- per-trial entry (src/qkd_ldpc_algorithm.cpp:1031-1119) ---------------
inline LDPC_result QKD_LDPC(const H_matrix &matrix, const std::vector<int> &alice_bit_array,
                            const std::vector<int> &bob_bit_array, const double &QBER,
                            const decoding_scaling_factors &scaling_factors = {},
                            const H_matrix_params &matrix_params = {}) {
    const size_t n = matrix.bit_nodes.size(), m = matrix.check_nodes.size();
    const double log_p = std::log((1. - QBER) / QBER);
    std::vector<double> apriori_llr(n);
    for (size_t i = 0; i < n; ++i) apriori_llr[i] = bob_bit_array[i] ? -log_p : log_p;
    std::vector<int> alice_syndrome(m);
    calculate_syndrome(alice_bit_array, matrix, alice_syndrome);
    std::vector<int> bob_solution(n);
    LDPC_result r;
    r.decoding_res = detail::decode_one((int32_t)CFG.DECODING_ALGORITHM, apriori_llr, matrix, alice_syndrome,
                                        CFG.DECODING_ALG_MAX_ITERATIONS, scaling_factors.primary,
                                        scaling_factors.secondary, CFG.DECODING_ALG_MSG_LLR_THRESHOLD, bob_solution);
    r.keys_match = arrays_equal(alice_bit_array, bob_solution);
    if (CFG.ENABLE_PRIVACY_MAINTENANCE) {
        std::vector<int> a_pm, b_pm;
        remove_bits(matrix_params.bits_to_remove, alice_bit_array, bob_solution, a_pm, b_pm);
    }
    return r;
}

// ---- batched entry for drivers ---------------------------------------------
// `batch` frames, frame-major: llr[batch*n], syndrome[batch*m] in {0,1}.
inline std::vector<decoding_result> decode_batch(const H_matrix &matrix, const std::vector<double> &llr,
                                                 const std::vector<uint8_t> &syndrome, size_t batch,
                                                 const decoding_scaling_factors &sf,
                                                 std::vector<uint8_t> &bits_out) {
    auto g = detail::graph_cache.get(matrix);
    const size_t n = matrix.bit_nodes.size();
    bits_out.resize(batch * n);
    std::vector<uint32_t> it(batch);
    std::vector<uint8_t> ok(batch);
    qldpc_params p{(int32_t)CFG.DECODING_ALGORITHM, (int32_t)CFG.DECODING_ALG_MAX_ITERATIONS,
                   CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD ? 1 : 0, 0, CFG.DECODING_ALG_MSG_LLR_THRESHOLD,
                   sf.primary, sf.secondary};
    if (qldpc_decode_batch(g.get(), &p, (int32_t)batch, llr.data(), syndrome.data(), bits_out.data(), it.data(),
                           ok.data(), nullptr))
        detail::raise("qldpc_decode_batch");
    std::vector<decoding_result> res(batch);
    for (size_t f = 0; f < batch; ++f) res[f] = {it[f], ok[f] != 0};
    return res;
}

}  // namespace qkd_ldpc_v_amd
