// simulation_batch.cpp — drop-in for the reference's QKD_LDPC_batch_simulation
// (ColdCloudd/QKD_LDPC_V src/simulation.cpp:693-760): the same simulation
// loop over matrices and combinations, the same per-trial seeds and the same
// statistics (its own process_trials_results, :580-690), with the trial loop
// — a BS::thread_pool running run_trial once per trial (:740-746) — replaced by
// ONE device batch per combination, sharded over the node's GPUs
// (qldpc_run_trials_submit / _wait: trials generated, frames built, decoded
// and compared on device; only the seeds go in and the per-trial results come
// out), combination c + 1 submitted before combination c is collected.
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
#include <exception>
#include <limits>
#include <memory>
#include <random>
#include <vector>

#include "../qkd_ldpc_impl.hpp"
#include "simulation_batch.hpp"

namespace {
namespace qi = qkd_ldpc_v_amd::impl;
}  // namespace

namespace {

// One combination on the GPUs: its trials submitted (qldpc_run_trials_submit),
// or the error run_trial would have thrown, raised when the loop reaches it.
struct Pending {
    std::unique_ptr<qi::TrialsJob> job;
    std::exception_ptr err;
};

Pending submit_combination(const H_matrix &matrix, double config_QBER, const std::vector<size_t> &seeds,
                           size_t curr_sim, const H_matrix_params &matrix_params,
                           const decoding_scaling_factors &scaling_factors) {
    const qi::DecodeConfig cfg{(int32_t)CFG.DECODING_ALGORITHM, (size_t)CFG.DECODING_ALG_MAX_ITERATIONS,
                               (bool)CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD,
                               (double)CFG.DECODING_ALG_MSG_LLR_THRESHOLD};
    const bool ra = CFG.ENABLE_CODE_RATE_ADAPTATION;  // run_trial's dispatch (:563-574)
    Pending p;
    try {
        p.job = qi::submit_trials(matrix, config_QBER, seeds, curr_sim, scaling_factors.primary,
                                  scaling_factors.secondary, cfg, ra ? &matrix_params.punctured_bits : nullptr,
                                  ra ? &matrix_params.shortened_bits : nullptr);
    } catch (...) {
        p.err = std::current_exception();
    }
    return p;
}

void collect(Pending &p, std::vector<trial_result> &trial_results) {
    if (p.err) std::rethrow_exception(p.err);
    const auto r = p.job->wait();
    const double q = p.job->accurate_qber();
    p.job.reset();
    trial_results.resize(r.size());
    for (size_t t = 0; t < r.size(); ++t) {
        trial_result &o = trial_results[t];
        o.ldpc_res.decoding_res.iterations_num = r[t].iterations_num;
        o.ldpc_res.decoding_res.syndromes_match = r[t].syndromes_match;
        o.ldpc_res.keys_match = r[t].keys_match;
        o.accurate_QBER = q;
        // trial_result::runtime is whole microseconds; a trial's share of a
        // GPU batch is a few, so it is rounded to nearest and kept >= 1 (the
        // throughput columns divide by it, :641-650).  The Python driver
        // applies the same rule (simulation.throughput_stats).
        o.runtime = std::chrono::microseconds(std::max<long long>(1, std::llround(r[t].runtime_us)));
    }
}

}  // namespace

void qkd_ldpc_hip_run_trials(const H_matrix &matrix, double config_QBER, const std::vector<size_t> &seeds,
                             size_t curr_sim, const H_matrix_params &matrix_params,
                             const decoding_scaling_factors &scaling_factors,
                             std::vector<trial_result> &trial_results) {
    Pending p = submit_combination(matrix, config_QBER, seeds, curr_sim, matrix_params, scaling_factors);
    collect(p, trial_results);
}

std::vector<sim_result> QKD_LDPC_batch_simulation(const std::vector<sim_input> &sim_in) {
    // the combinations in the reference's order (matrix by matrix, :725-730)
    std::vector<std::pair<const sim_input *, const sim_combination *>> combos;
    for (const auto &in : sim_in)
        for (const auto &comb : in.combinations) combos.push_back({&in, &comb});
    std::vector<sim_result> sim_results(combos.size());
    std::vector<trial_result> trial_results(CFG.TRIALS_NUMBER);
    // the per-trial seeds, drawn once for the whole run (:713-719)
    std::vector<size_t> seeds(CFG.TRIALS_NUMBER);
    {
        XoshiroCpp::Xoshiro256PlusPlus prng(CFG.SIMULATION_SEED);
        std::uniform_int_distribution<size_t> draw(0, std::numeric_limits<size_t>::max());
        std::generate(seeds.begin(), seeds.end(), [&] { return draw(prng); });
    }
    auto submit = [&](size_t sim) {
        const sim_combination &comb = *combos[sim].second;
        return submit_combination(combos[sim].first->matrix, comb.config_QBER, seeds, sim, comb.matrix_params,
                                  comb.scaling_factors);
    };
    // combination c + 1 goes onto the GPUs before combination c is collected,
    // so its trial generation runs while c's last frames decode
    Pending next;
    if (!combos.empty()) next = submit(0);
    for (size_t curr_sim = 0; curr_sim < combos.size(); ++curr_sim) {
        Pending cur = std::move(next);
        if (curr_sim + 1 < combos.size()) next = submit(curr_sim + 1);
        collect(cur, trial_results);
        const sim_input &in = *combos[curr_sim].first;
        const H_matrix &matrix = in.matrix;
        const sim_combination &comb = *combos[curr_sim].second;
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
    }
    return sim_results;
}
