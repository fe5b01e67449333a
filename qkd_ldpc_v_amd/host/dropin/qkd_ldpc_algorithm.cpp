// qkd_ldpc_algorithm.cpp — drop-in replacement for the reference's
// src/qkd_ldpc_algorithm.cpp (ColdCloudd/QKD_LDPC_V): every function its
// header declares (src/qkd_ldpc_algorithm.hpp:28-109), with the same
// signatures, defined on libqkdldpc_hip.so.  The reference's build compiles
// this file INSTEAD of src/qkd_ldpc_algorithm.cpp:
//
//   g++ -std=c++20 -I src -I <this repo>/include ...
//       <this repo>/qkd_ldpc_v_amd/host/dropin/qkd_ldpc_algorithm.cpp
//       -L<this repo>/qkd_ldpc_v_amd -lqkdldpc_hip
//
// so "qkd_ldpc_algorithm.hpp" below is the reference's own header, and CFG,
// H_matrix, decoding_scaling_factors, H_matrix_params, DEC_* and
// XoshiroCpp::Xoshiro256PlusPlus are the reference's own declarations
// (src/config.hpp:50-54,198-203; src/array_and_matrix_operations.hpp:27-77).
// The hidden inputs are read from CFG exactly where the reference reads them:
// DECODING_ALGORITHM / DECODING_ALG_MAX_ITERATIONS / DECODING_ALG_MSG_LLR_THRESHOLD
// in QKD_LDPC / QKD_LDPC_RATE_ADAPT (:1056-1085, :1185-1214) and
// ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD inside every decoder.  The TRACE_*
// console output is not reproduced (tracing is off the GPU path).
// Device graphs are cached by H content (qkd_ldpc_impl.hpp GraphCache): the
// reference hands the same H to every trial of a combination.
#include "qkd_ldpc_algorithm.hpp"

#include "../qkd_ldpc_impl.hpp"

namespace {

namespace qi = qkd_ldpc_v_amd::impl;

qi::DecodeConfig hot_cfg() {
    return {(int32_t)CFG.DECODING_ALGORITHM, (size_t)CFG.DECODING_ALG_MAX_ITERATIONS,
            (bool)CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD, (double)CFG.DECODING_ALG_MSG_LLR_THRESHOLD};
}

decoding_result run(int32_t alg, const std::vector<double> &llr, const H_matrix &H, const std::vector<int> &syndrome,
                    size_t max_it, double primary, double secondary, double thr, std::vector<int> &out) {
    const auto r = qi::decode_one(alg, llr, H, syndrome, max_it, primary, secondary,
                                  (bool)CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD, thr, out);
    decoding_result d;
    d.iterations_num = r.first;
    d.syndromes_match = r.second;
    return d;
}

LDPC_result to_ldpc(const qi::TrialResult &r) {
    LDPC_result o;
    o.decoding_res.iterations_num = r.iterations_num;
    o.decoding_res.syndromes_match = r.syndromes_match;
    o.keys_match = r.keys_match;
    return o;
}

}  // namespace

decoding_result sum_product_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                     const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                     const double &msg_threshold, std::vector<int> &bit_array_out) {
    return run(QLDPC_SPA, bit_array_llr, matrix, syndrome, max_num_iterations, 0, 0, msg_threshold, bit_array_out);
}

double tanh_lin_approx(double x) { return qi::tanh_lin_approx(x); }

double atanh_lin_approx(double x) { return qi::atanh_lin_approx(x); }

decoding_result sum_product_linear_approx_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                                   const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                                   const double &msg_threshold, std::vector<int> &bit_array_out) {
    return run(QLDPC_SPA_LIN, bit_array_llr, matrix, syndrome, max_num_iterations, 0, 0, msg_threshold,
               bit_array_out);
}

decoding_result min_sum_normalized_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                            const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                            const double &alpha, const double &msg_threshold,
                                            std::vector<int> &bit_array_out) {
    return run(QLDPC_NMSA, bit_array_llr, matrix, syndrome, max_num_iterations, alpha, 0, msg_threshold,
               bit_array_out);
}

decoding_result min_sum_offset_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                        const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                        const double &beta, const double &msg_threshold,
                                        std::vector<int> &bit_array_out) {
    return run(QLDPC_OMSA, bit_array_llr, matrix, syndrome, max_num_iterations, beta, 0, msg_threshold,
               bit_array_out);
}

decoding_result adaptive_min_sum_normalized_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                                     const std::vector<int> &syndrome,
                                                     const size_t &max_num_iterations, const double &alpha,
                                                     const double &nu, const double &msg_threshold,
                                                     std::vector<int> &bit_array_out) {
    return run(QLDPC_ANMSA, bit_array_llr, matrix, syndrome, max_num_iterations, alpha, nu, msg_threshold,
               bit_array_out);
}

decoding_result adaptive_min_sum_offset_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                                 const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                                 const double &beta, const double &sigma,
                                                 const double &msg_threshold, std::vector<int> &bit_array_out) {
    return run(QLDPC_AOMSA, bit_array_llr, matrix, syndrome, max_num_iterations, beta, sigma, msg_threshold,
               bit_array_out);
}

LDPC_result QKD_LDPC(const H_matrix &matrix, const std::vector<int> &alice_bit_array,
                     const std::vector<int> &bob_bit_array, const double &QBER,
                     const decoding_scaling_factors &scaling_factors, const H_matrix_params &matrix_params) {
    (void)matrix_params;  // privacy maintenance's remove_bits only feeds the TRACE output (:1089-1092)
    return to_ldpc(qi::qkd_ldpc(matrix, alice_bit_array, bob_bit_array, QBER, scaling_factors.primary,
                                scaling_factors.secondary, hot_cfg()));
}

LDPC_result QKD_LDPC_RATE_ADAPT(const H_matrix &matrix, const std::vector<int> &alice_bit_array,
                                const std::vector<int> &bob_bit_array, const double &QBER,
                                const decoding_scaling_factors &scaling_factors, const H_matrix_params &matrix_params,
                                XoshiroCpp::Xoshiro256PlusPlus &prng) {
    return to_ldpc(qi::qkd_ldpc_rate_adapt(matrix, alice_bit_array, bob_bit_array, QBER, scaling_factors.primary,
                                           scaling_factors.secondary, matrix_params.punctured_bits,
                                           matrix_params.shortened_bits, prng, hot_cfg()));
}
