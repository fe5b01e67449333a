// qkd_ldpc_algorithm.hpp — C++ mirror of the reference's decode interface in
// namespace qkd_ldpc_v_amd, backed by libqkdldpc_hip.so (include/qkd_ldpc_hip.h).
//
// Same names, argument meaning and error behaviour as ColdCloudd/QKD_LDPC_V:
//   H_matrix, H_matrix_params src/array_and_matrix_operations.hpp:27-77
//   read_sparse_*             src/array_and_matrix_operations.cpp:291-886
//   decoding_result, LDPC_result, the six decoders, tanh/atanh_lin_approx,
//   QKD_LDPC, QKD_LDPC_RATE_ADAPT
//                             src/qkd_ldpc_algorithm.hpp:16-109
//   calculate_syndrome, arrays_equal, remove_bits
//                             src/array_and_matrix_operations.cpp:105-118,259-287,936-950
//   config_data / CFG (the subset the hot path reads)   src/config.hpp:103-198
// For a program that includes this header instead of the reference's.  The
// drop-in for the reference's OWN build — its globals, its H_matrix, its
// generator type — is dropin/qkd_ldpc_algorithm.cpp; both
// are thin layers over qkd_ldpc_impl.hpp.  decode_batch() is the batched entry
// a driver uses in place of the per-trial thread pool (src/simulation.cpp:740-746).
// Errors are std::runtime_error carrying qldpc_last_error().
#pragma once

#include <cmath>
#include <cstdint>
#include <filesystem>
#include <stdexcept>
#include <string>
#include <vector>

#include "qkd_ldpc_hip.h"
#include "qkd_ldpc_impl.hpp"

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
    bool ENABLE_CODE_RATE_ADAPTATION{};
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

inline impl::DecodeConfig cfg() {
    return {(int32_t)CFG.DECODING_ALGORITHM, CFG.DECODING_ALG_MAX_ITERATIONS, CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD,
            CFG.DECODING_ALG_MSG_LLR_THRESHOLD};
}

inline decoding_result decode(int32_t alg, const std::vector<double> &llr, const H_matrix &H,
                              const std::vector<int> &syndrome, size_t max_it, double primary, double secondary,
                              double thr, std::vector<int> &out) {
    const auto r = impl::decode_one(alg, llr, H, syndrome, max_it, primary, secondary,
                                    CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD, thr, out);
    return {r.first, r.second};
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
    impl::calculate_syndrome(bit_array, matrix, syndrome_out);
}
inline bool arrays_equal(const std::vector<int> &a, const std::vector<int> &b) { return impl::arrays_equal(a, b); }
inline void remove_bits(const std::vector<int> &bits_to_remove, const std::vector<int> &array1,
                        const std::vector<int> &array2, std::vector<int> &array1_out, std::vector<int> &array2_out) {
    impl::remove_bits(bits_to_remove, array1, array2, array1_out, array2_out);
}

// ---- the six decoders and the linear approximations (src/qkd_ldpc_algorithm.hpp:28-90)
inline decoding_result sum_product_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                            const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                            const double &msg_threshold, std::vector<int> &bit_array_out) {
    return detail::decode(QLDPC_SPA, bit_array_llr, matrix, syndrome, max_num_iterations, 0, 0, msg_threshold,
                          bit_array_out);
}
inline double tanh_lin_approx(double x) { return impl::tanh_lin_approx(x); }
inline double atanh_lin_approx(double x) { return impl::atanh_lin_approx(x); }
inline decoding_result sum_product_linear_approx_decoding(const std::vector<double> &bit_array_llr,
                                                          const H_matrix &matrix, const std::vector<int> &syndrome,
                                                          const size_t &max_num_iterations,
                                                          const double &msg_threshold,
                                                          std::vector<int> &bit_array_out) {
    return detail::decode(QLDPC_SPA_LIN, bit_array_llr, matrix, syndrome, max_num_iterations, 0, 0, msg_threshold,
                          bit_array_out);
}
inline decoding_result min_sum_normalized_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                                   const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                                   const double &alpha, const double &msg_threshold,
                                                   std::vector<int> &bit_array_out) {
    return detail::decode(QLDPC_NMSA, bit_array_llr, matrix, syndrome, max_num_iterations, alpha, 0, msg_threshold,
                          bit_array_out);
}
inline decoding_result min_sum_offset_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                               const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                               const double &beta, const double &msg_threshold,
                                               std::vector<int> &bit_array_out) {
    return detail::decode(QLDPC_OMSA, bit_array_llr, matrix, syndrome, max_num_iterations, beta, 0, msg_threshold,
                          bit_array_out);
}
inline decoding_result adaptive_min_sum_normalized_decoding(const std::vector<double> &bit_array_llr,
                                                            const H_matrix &matrix, const std::vector<int> &syndrome,
                                                            const size_t &max_num_iterations, const double &alpha,
                                                            const double &nu, const double &msg_threshold,
                                                            std::vector<int> &bit_array_out) {
    return detail::decode(QLDPC_ANMSA, bit_array_llr, matrix, syndrome, max_num_iterations, alpha, nu, msg_threshold,
                          bit_array_out);
}
inline decoding_result adaptive_min_sum_offset_decoding(const std::vector<double> &bit_array_llr,
                                                        const H_matrix &matrix, const std::vector<int> &syndrome,
                                                        const size_t &max_num_iterations, const double &beta,
                                                        const double &sigma, const double &msg_threshold,
                                                        std::vector<int> &bit_array_out) {
    return detail::decode(QLDPC_AOMSA, bit_array_llr, matrix, syndrome, max_num_iterations, beta, sigma,
                          msg_threshold, bit_array_out);
}

// ---- per-trial entries (src/qkd_ldpc_algorithm.cpp:1031-1258) --------------
inline LDPC_result QKD_LDPC(const H_matrix &matrix, const std::vector<int> &alice_bit_array,
                            const std::vector<int> &bob_bit_array, const double &QBER,
                            const decoding_scaling_factors &scaling_factors = {},
                            const H_matrix_params &matrix_params = {}) {
    (void)matrix_params;  // privacy maintenance's remove_bits only feeds the reference's TRACE output
    const auto r = impl::qkd_ldpc(matrix, alice_bit_array, bob_bit_array, QBER, scaling_factors.primary,
                                  scaling_factors.secondary, detail::cfg());
    return {{r.iterations_num, r.syndromes_match}, r.keys_match};
}

// The reference takes XoshiroCpp::Xoshiro256PlusPlus&; any uniform random bit
// generator binds here, and its draws are consumed exactly as there (two
// uniform_int_distribution<int>(0, 1) draws per punctured position, in
// position order).
template <class URBG>
LDPC_result QKD_LDPC_RATE_ADAPT(const H_matrix &matrix, const std::vector<int> &alice_bit_array,
                                const std::vector<int> &bob_bit_array, const double &QBER,
                                const decoding_scaling_factors &scaling_factors, const H_matrix_params &matrix_params,
                                URBG &prng) {
    const auto r = impl::qkd_ldpc_rate_adapt(matrix, alice_bit_array, bob_bit_array, QBER, scaling_factors.primary,
                                             scaling_factors.secondary, matrix_params.punctured_bits,
                                             matrix_params.shortened_bits, prng, detail::cfg());
    return {{r.iterations_num, r.syndromes_match}, r.keys_match};
}

// ---- batched entry for drivers ---------------------------------------------
// `batch` frames, frame-major: llr[batch*n], syndrome[batch*m] in {0,1}.
inline std::vector<decoding_result> decode_batch(const H_matrix &matrix, const std::vector<double> &llr,
                                                 const std::vector<uint8_t> &syndrome, size_t batch,
                                                 const decoding_scaling_factors &sf,
                                                 std::vector<uint8_t> &bits_out) {
    auto e = impl::graph_cache().get(matrix);
    const size_t n = matrix.bit_nodes.size(), m = matrix.check_nodes.size();
    if (llr.size() < batch * n || syndrome.size() < batch * m)
        throw std::runtime_error("decode_batch: llr / syndrome shorter than batch frames");
    bits_out.resize(batch * n);
    std::vector<uint32_t> it(batch);
    std::vector<uint8_t> ok(batch);
    qldpc_params p{(int32_t)CFG.DECODING_ALGORITHM, (int32_t)CFG.DECODING_ALG_MAX_ITERATIONS,
                   CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD ? 1 : 0, 0, CFG.DECODING_ALG_MSG_LLR_THRESHOLD,
                   sf.primary, sf.secondary};
    if (qldpc_decode_batch(e->g.get(), &p, (int32_t)batch, llr.data(), syndrome.data(), bits_out.data(), it.data(),
                           ok.data(), nullptr))
        impl::raise("qldpc_decode_batch");
    std::vector<decoding_result> res(batch);
    for (size_t f = 0; f < batch; ++f) res[f] = {it[f], ok[f] != 0};
    return res;
}

// The simulation loop's batch seam: run_trial for every seed of one
// combination (src/simulation.cpp:540-576, 721-746; trial t seeded with
// seeds[t] + seed_add), on the GPUs the cached graph lives on.  With
// CFG.ENABLE_CODE_RATE_ADAPTATION the trials run QKD_LDPC_RATE_ADAPT with
// matrix_params' punctured / shortened positions, else QKD_LDPC.
struct trial_result {  // src/simulation.hpp:36-41 (runtime in microseconds, as a double)
    LDPC_result ldpc_res{};
    double accurate_QBER{};
    double runtime_us{};
};
inline std::vector<trial_result> run_trials(const H_matrix &matrix, double QBER, const std::vector<size_t> &seeds,
                                            size_t seed_add, const H_matrix_params &matrix_params = {},
                                            const decoding_scaling_factors &sf = {}) {
    const bool ra = CFG.ENABLE_CODE_RATE_ADAPTATION;
    double q = 0.;
    const auto r = impl::run_trials(matrix, QBER, seeds, seed_add, sf.primary, sf.secondary, detail::cfg(),
                                    ra ? &matrix_params.punctured_bits : nullptr,
                                    ra ? &matrix_params.shortened_bits : nullptr, &q);
    std::vector<trial_result> out(r.size());
    for (size_t t = 0; t < r.size(); ++t) out[t] = {{{r[t].iterations_num, r[t].syndromes_match}, r[t].keys_match}, q,
                                                    r[t].runtime_us};
    return out;
}

// Device graphs are cached by H content; free one (or all) explicitly.
inline bool release_matrix(const H_matrix &matrix) { return impl::graph_cache().release(matrix); }
inline void release_all_matrices() { impl::graph_cache().clear(); }

}  // namespace qkd_ldpc_v_amd
