// simulation_batch.hpp — the batch seam of the reference's simulation loop,
// as the drop-in TU simulation_batch.cpp defines it for the reference's own
// build.  Include after the reference's "simulation.hpp".
#pragma once

#include <cstddef>
#include <vector>

// One combination's trials (the body of QKD_LDPC_batch_simulation's
// pool.detach_loop(0, TRIALS_NUMBER), src/simulation.cpp:740-746):
// trial_results[n] = run_trial(matrix, config_QBER, seeds[n] + curr_sim,
// matrix_params, scaling_factors) for every n, computed as ONE batch on the
// GPUs of the node (qldpc_run_trials) — keys generated, frames built, decoded
// and compared on device.  trial_results is resized to seeds.size().
void qkd_ldpc_hip_run_trials(const H_matrix &matrix, double config_QBER, const std::vector<size_t> &seeds,
                             size_t curr_sim, const H_matrix_params &matrix_params,
                             const decoding_scaling_factors &scaling_factors,
                             std::vector<trial_result> &trial_results);
