// simulation_batch.cpp — drop-in for the reference's QKD_LDPC_batch_simulation
// (ColdCloudd/QKD_LDPC_V src/simulation.cpp:693-760): the same simulation
// loop over matrices and combinations, the same per-trial seeds and the same
// statistics (its own process_trials_results, :580-690), with the trial loop
// — a BS::thread_pool running run_trial once per trial (:740-746) — replaced by
// ONE device batch per combination, sharded over the node's GPUs
// (qldpc_run_trials: trials generated, frames built, decoded and compared on
// device; only the seeds go in and the per-trial results come out).
//
// The reference's build compiles this file beside dropin/qkd_ldpc_algorithm.cpp
// and drops its own definition of QKD_LDPC_batch_simulation (INTEGRATION.md
// §3), so "simulation.hpp" below is the reference's own header and sim_input,
// sim_result, trial_result, process_trials_results and CFG are its
// declarations.  The GPUs: QKD_LDPC_HIP_DEVICES (a comma list) or all.  The
// console progress bar is not reproduced (out of the hot path).
#include "simulation.hpp"

#include <algorithm>
#include <cmath>
#include <limits>
#include <random>
#include <vector>

#include "../qkd_ldpc_impl.hpp"
#include "simulation_batch.hpp"

namespace {
namespace qi = qkd_ldpc_v_amd::impl;
}  // namespace

void qkd_ldpc_hip_run_trials(const H_matrix &matrix, double config_QBER, const std::vector<size_t> &seeds,
                             size_t curr_sim, const H_matrix_params &matrix_params,
                             const decoding_scaling_factors &scaling_factors,
                             std::vector<trial_result> &trial_results) {
    const qi::DecodeConfig cfg{(int32_t)CFG.DECODING_ALGORITHM, (size_t)CFG.DECODING_ALG_MAX_ITERATIONS,
                               (bool)CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD,
                               (double)CFG.DECODING_ALG_MSG_LLR_THRESHOLD};
    const bool ra = CFG.ENABLE_CODE_RATE_ADAPTATION;  // run_trial's dispatch (:563-574)
    double q = 0.;
    const auto r = qi::run_trials(matrix, config_QBER, seeds, curr_sim, scaling_factors.primary,
                                  scaling_factors.secondary, cfg, ra ? &matrix_params.punctured_bits : nullptr,
                                  ra ? &matrix_params.shortened_bits : nullptr, &q);
    trial_results.resize(r.size());
    for (size_t t = 0; t < r.size(); ++t) {
        trial_result &o = trial_results[t];
        o.ldpc_res.decoding_res.iterations_num = r[t].iterations_num;
        o.ldpc_res.decoding_res.syndromes_match = r[t].syndromes_match;
        o.ldpc_res.keys_match = r[t].keys_match;
        o.accurate_QBER = q;
        // trial_result::runtime is whole microseconds; a trial's share of a
        // GPU batch is a few, so it is rounded to nearest and kept >= 1 (the
        // throughput columns divide by it, :641-650)
        o.runtime = std::chrono::microseconds(std::max<long long>(1, std::llround(r[t].runtime_us)));
    }
}

std::vector<sim_result> QKD_LDPC_batch_simulation(const std::vector<sim_input> &sim_in) {
    size_t sim_total = 0;
    for (const auto &in : sim_in) sim_total += in.combinations.size();
    std::vector<sim_result> sim_results(sim_total);
    std::vector<trial_result> trial_results(CFG.TRIALS_NUMBER);
    // the per-trial seeds, drawn once for the whole run (:713-719)
    std::vector<size_t> seeds(CFG.TRIALS_NUMBER);
    {
        XoshiroCpp::Xoshiro256PlusPlus prng(CFG.SIMULATION_SEED);
        std::uniform_int_distribution<size_t> draw(0, std::numeric_limits<size_t>::max());
        std::generate(seeds.begin(), seeds.end(), [&] { return draw(prng); });
    }
    size_t curr_sim = 0;
    for (const sim_input &in : sim_in) {
        const H_matrix &matrix = in.matrix;
        for (const sim_combination &comb : in.combinations) {
            qkd_ldpc_hip_run_trials(matrix, comb.config_QBER, seeds, curr_sim, comb.matrix_params,
                                    comb.scaling_factors, trial_results);
            const H_matrix_params &mp = comb.matrix_params;
            sim_result &res = sim_results[curr_sim];
            res.sim_number = curr_sim;
            res.matrix_filename = in.matrix_path.filename().string();
            res.is_regular = matrix.is_regular;
            res.num_bit_nodes = matrix.bit_nodes.size();
            res.num_check_nodes = matrix.check_nodes.size();
            res.delta = mp.delta;
            res.efficiency = mp.efficiency;
            res.punctured_fraction = mp.punctured_fraction;
            res.shortened_fraction = mp.shortened_fraction;
            res.adapted_code_rate = mp.adapted_code_rate;
            res.config_QBER = comb.config_QBER;
            res.accurate_QBER = trial_results.empty() ? 0. : trial_results[0].accurate_QBER;
            res.scaling_factors = comb.scaling_factors;
            process_trials_results(trial_results, matrix, mp, res);  // the reference's own statistics
            ++curr_sim;
        }
    }
    return sim_results;
}
