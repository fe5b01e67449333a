// The simulation-loop interface dropin/simulation_batch.cpp binds to, declared
// for the drop-in test: the names, members and signatures of the reference's
// src/simulation.hpp:22-120 (sim_combination, sim_input, trial_result,
// sim_result, run_trial, process_trials_results, QKD_LDPC_batch_simulation),
// in the global namespace as there.  Written for this test from those
// declarations (the reference's header also pulls fmt, BS_thread_pool and
// indicators, absent here); it is not the reference's header.
#pragma once

#include <chrono>
#include <filesystem>
#include <string>
#include <vector>

#include "qkd_ldpc_algorithm.hpp"

namespace fs = std::filesystem;

struct sim_combination {
    double config_QBER;
    H_matrix_params matrix_params;
    decoding_scaling_factors scaling_factors;
};

struct sim_input {
    H_matrix matrix{};
    fs::path matrix_path{};
    std::vector<sim_combination> combinations;
};

struct trial_result {
    LDPC_result ldpc_res{};
    double accurate_QBER{};
    std::chrono::microseconds runtime{};
};

struct sim_result {
    size_t sim_number{};
    std::string matrix_filename{};
    bool is_regular{};
    size_t num_bit_nodes{};
    size_t num_check_nodes{};
    double delta{};
    double efficiency{};
    double punctured_fraction{};
    double shortened_fraction{};
    double adapted_code_rate{};
    double config_QBER;
    double accurate_QBER{};
    decoding_scaling_factors scaling_factors{};
    size_t iter_success_dec_alg_max{};
    size_t iter_success_dec_alg_min{};
    double iter_success_dec_alg_mean{};
    double iter_success_dec_alg_std_dev{};
    double ratio_trials_success_dec_alg{};
    double ratio_trials_success_ldpc{};
    size_t throughput_max{};
    size_t throughput_min{};
    size_t throughput_mean{};
    size_t throughput_std_dev{};
};

trial_result run_trial(const H_matrix &matrix, double QBER, size_t seed, const H_matrix_params &matrix_params = {},
                       const decoding_scaling_factors &scaling_factors = {});

void process_trials_results(const std::vector<trial_result> &trial_results, const H_matrix &matrix,
                            const H_matrix_params &matrix_params, sim_result &result);

std::vector<sim_result> QKD_LDPC_batch_simulation(const std::vector<sim_input> &sim_in);
