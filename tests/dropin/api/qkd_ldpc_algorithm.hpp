// The interface dropin/qkd_ldpc_algorithm.cpp binds to, declared for the
// drop-in test: the names, members and signatures the reference's headers
// give them (src/qkd_ldpc_algorithm.hpp:13-109, src/config.hpp:50-54,103-203,
// src/array_and_matrix_operations.hpp:27-77), in the global namespace as
// there.  Written for this test from those declarations; it is not the
// reference's header (which also pulls fmt, nlohmann::json and the absent
// Xoshiro-cpp package): the test compiles the replacement translation unit
// against it exactly as the reference's build compiles it against src/.
#pragma once

#include <cstddef>
#include <cstdint>
#include <limits>
#include <vector>

// The generator type of the reference's trials (Xoshiro-cpp v1.1's
// Xoshiro256PlusPlus: SplitMix64 seeding, rotl(s0 + s3, 23) + s0), as a
// UniformRandomBitGenerator.
namespace XoshiroCpp {
class Xoshiro256PlusPlus {
  public:
    using result_type = uint64_t;
    explicit Xoshiro256PlusPlus(uint64_t seed) {
        uint64_t x = seed;
        for (auto &v : s_) {
            uint64_t z = (x += 0x9e3779b97f4a7c15ull);
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
            v = z ^ (z >> 31);
        }
    }
    static constexpr result_type min() { return 0; }
    static constexpr result_type max() { return std::numeric_limits<uint64_t>::max(); }
    result_type operator()() {
        const uint64_t r = rotl(s_[0] + s_[3], 23) + s_[0];
        const uint64_t t = s_[1] << 17;
        s_[2] ^= s_[0];
        s_[3] ^= s_[1];
        s_[1] ^= s_[2];
        s_[0] ^= s_[3];
        s_[2] ^= t;
        s_[3] = rotl(s_[3], 45);
        return r;
    }

  private:
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t s_[4];
};
}  // namespace XoshiroCpp

struct decoding_scaling_factors {
    double primary{};
    double secondary{};
};

struct config_data {  // the members the decode path and run_trial read
    size_t THREADS_NUMBER{};
    size_t TRIALS_NUMBER{};
    size_t SIMULATION_SEED{};
    bool ENABLE_PRIVACY_MAINTENANCE{};
    bool ENABLE_THROUGHPUT_MEASUREMENT{};
    bool CONSIDER_RTT{};
    double RTT{};
    size_t DECODING_ALGORITHM{};
    size_t DECODING_ALG_MAX_ITERATIONS{};
    size_t MATRIX_FORMAT{};
    bool TRACE_QKD_LDPC{};
    bool TRACE_DECODING_ALG{};
    bool TRACE_DECODING_ALG_LLR{};
    bool ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD{};
    double DECODING_ALG_MSG_LLR_THRESHOLD{};
    bool ENABLE_CODE_RATE_ADAPTATION{};
    bool ENABLE_UNTAINTED_PUNCTURING{};
};
extern config_data CFG;

inline constexpr size_t DEC_SPA = 0, DEC_SPA_APPROX = 1, DEC_NMSA = 2, DEC_OMSA = 3, DEC_ANMSA = 4, DEC_AOMSA = 5;
inline constexpr size_t MAT_SPARSE_UNCOMPRESSED = 0, MAT_SPARSE_ALIST = 1, MAT_SPARSE_1 = 2, MAT_SPARSE_2 = 3;

struct H_matrix_params {
    double delta{};
    double efficiency{};
    double punctured_fraction{};
    double shortened_fraction{};
    double adapted_code_rate{};
    std::vector<int> punctured_bits{};
    std::vector<int> shortened_bits{};
    std::vector<int> bits_to_remove{};
};

struct H_matrix {
    std::vector<std::vector<int>> bit_nodes{};
    std::vector<std::vector<int>> check_nodes{};
    std::vector<int> punctured_bits_untainted{};
    bool is_regular{};
};

const double ALMOST_ZERO = 1e-4;

struct decoding_result {
    size_t iterations_num{};
    bool syndromes_match{};
};

struct LDPC_result {
    decoding_result decoding_res{};
    bool keys_match{};
};

decoding_result sum_product_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                     const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                     const double &msg_threshold, std::vector<int> &bit_array_out);
double tanh_lin_approx(double x);
double atanh_lin_approx(double x);
decoding_result sum_product_linear_approx_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                                   const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                                   const double &msg_threshold, std::vector<int> &bit_array_out);
decoding_result min_sum_normalized_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                            const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                            const double &alpha, const double &msg_threshold,
                                            std::vector<int> &bit_array_out);
decoding_result min_sum_offset_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                        const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                        const double &beta, const double &msg_threshold,
                                        std::vector<int> &bit_array_out);
decoding_result adaptive_min_sum_normalized_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                                     const std::vector<int> &syndrome,
                                                     const size_t &max_num_iterations, const double &alpha,
                                                     const double &nu, const double &msg_threshold,
                                                     std::vector<int> &bit_array_out);
decoding_result adaptive_min_sum_offset_decoding(const std::vector<double> &bit_array_llr, const H_matrix &matrix,
                                                 const std::vector<int> &syndrome, const size_t &max_num_iterations,
                                                 const double &beta, const double &sigma,
                                                 const double &msg_threshold, std::vector<int> &bit_array_out);
LDPC_result QKD_LDPC(const H_matrix &matrix, const std::vector<int> &alice_bit_array,
                     const std::vector<int> &bob_bit_array, const double &QBER,
                     const decoding_scaling_factors &scaling_factors = {}, const H_matrix_params &matrix_params = {});
LDPC_result QKD_LDPC_RATE_ADAPT(const H_matrix &matrix, const std::vector<int> &alice_bit_array,
                                const std::vector<int> &bob_bit_array, const double &QBER,
                                const decoding_scaling_factors &scaling_factors, const H_matrix_params &matrix_params,
                                XoshiroCpp::Xoshiro256PlusPlus &prng);
