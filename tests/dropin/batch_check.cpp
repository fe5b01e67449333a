// batch_check — the reference's simulation loop over the drop-in TUs
// (qkd_ldpc_v_amd/host/dropin/simulation_batch.cpp + qkd_ldpc_algorithm.cpp),
// compiled against the reference-shaped declarations in tests/dropin/api/.
// Test infrastructure (tests/test_dropin.py): run_trial and
// process_trials_results are restated here from src/simulation.cpp:540-690,
// as the reference's simulation.cpp provides them to the drop-in.
//
//   batch_check batch <matrix> <fmt> <alg> <primary> <secondary> <qbers.txt> <max_it> <trials> <sim_seed>
//                     <threads> [<punctured.txt> <shortened.txt>]
//       one sim_input with one combination per QBER (rate adaptation on when
//       position lists are given).  Prints, per combination `sim` and trial t:
//         "S sim t it ok km runtime_us"  the batch seam (qkd_ldpc_hip_run_trials)
//         "T sim t it ok km"             run_trial through the per-trial drop-in,
//                                        called from <threads> concurrent threads
//       then QKD_LDPC_batch_simulation's results:
//         "R sim dec ldpc it_max it_min it_mean it_std accurate_qber tp_mean tp_std tp_min tp_max"
//       and the wall times "W seam <s>" / "W pertrial <s>".
//   batch_check time <matrix> <fmt> <alg> <primary> <secondary> <qber> <max_it> <trials> <sim_seed> <threads>
//       throughput of one combination (decoded info bits n - m per trial):
//         "seam <trials> <seconds> <bits/s>" and "pertrial <trials> <seconds> <bits/s>"
//       (threads 0: the seam only)
//   batch_check sweep <matrix> <fmt> <alg> <primary> <secondary> <qbers.txt> <max_it> <trials> <sim_seed>
//                     [<punctured.txt> <shortened.txt>]
//       QKD_LDPC_batch_simulation over one combination per QBER (after a
//       two-combination warm-up), timed as a whole:
//         "sweep <combinations> <trials> <seconds> <ms per combination> <mean FER>"
// Failures print "ERROR: <what>" and exit 1.
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <limits>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "qkd_ldpc_algorithm.hpp"  // tests/dropin/api
#include "qkd_ldpc_hip.h"
#include "simulation.hpp"          // tests/dropin/api
#include "simulation_batch.hpp"    // qkd_ldpc_v_amd/host/dropin
#include "trial_common.hpp"

config_data CFG;  // defined by the reference's src/config.cpp

using namespace trial_common;

// run_trial (src/simulation.cpp:540-576), restated.
trial_result run_trial(const H_matrix &matrix, double QBER, size_t seed, const H_matrix_params &matrix_params,
                       const decoding_scaling_factors &scaling_factors) {
    trial_result result;
    XoshiroCpp::Xoshiro256PlusPlus prng(seed);
    const size_t n = matrix.bit_nodes.size();
    std::vector<int> alice(n), bob(n);
    fill_random_bits(prng, alice);
    result.accurate_QBER = inject_errors(prng, alice, QBER, bob);
    if (result.accurate_QBER == 0.)
        throw std::runtime_error("Key size '" + std::to_string(n) + "' is too small for QBER.");
    const auto t0 = std::chrono::high_resolution_clock::now();
    if (CFG.ENABLE_CODE_RATE_ADAPTATION)
        result.ldpc_res = QKD_LDPC_RATE_ADAPT(matrix, alice, bob, result.accurate_QBER, scaling_factors, matrix_params,
                                              prng);
    else
        result.ldpc_res = QKD_LDPC(matrix, alice, bob, result.accurate_QBER, scaling_factors, matrix_params);
    if (CFG.ENABLE_THROUGHPUT_MEASUREMENT)
        result.runtime = std::chrono::duration_cast<std::chrono::microseconds>(
            std::chrono::high_resolution_clock::now() - t0);
    return result;
}

// process_trials_results (src/simulation.cpp:580-690), restated: iteration
// statistics over the trials whose syndromes matched, success ratios over
// TRIALS_NUMBER, per-trial throughput out_key_length / runtime.
void process_trials_results(const std::vector<trial_result> &trial_results, const H_matrix &matrix,
                            const H_matrix_params &matrix_params, sim_result &result) {
    size_t ok = 0, keys = 0, it_max = 0, it_min = std::numeric_limits<size_t>::max();
    double it_mean = 0., it_std = 0.;
    for (const auto &t : trial_results) {
        if (!t.ldpc_res.decoding_res.syndromes_match) continue;
        const size_t it = t.ldpc_res.decoding_res.iterations_num;
        ++ok;
        it_max = std::max(it_max, it);
        it_min = std::min(it_min, it);
        if (t.ldpc_res.keys_match) ++keys;
        it_mean += (double)it;
    }
    if (ok > 0) {
        it_mean /= (double)ok;
        for (const auto &t : trial_results)
            if (t.ldpc_res.decoding_res.syndromes_match)
                it_std += std::pow((double)t.ldpc_res.decoding_res.iterations_num - it_mean, 2);
        it_std = std::sqrt(it_std / (double)ok);
    }
    if (CFG.ENABLE_THROUGHPUT_MEASUREMENT) {
        const size_t n = matrix.bit_nodes.size();
        const double out_len = (CFG.ENABLE_CODE_RATE_ADAPTATION || CFG.ENABLE_PRIVACY_MAINTENANCE)
                                   ? (double)(n - matrix_params.bits_to_remove.size())
                                   : (double)n;
        auto tp_of = [&](const trial_result &t) {
            const double us = (double)t.runtime.count() + (CFG.CONSIDER_RTT ? CFG.RTT * 1000. : 0.);
            return out_len * 1e6 / us;
        };
        double mx = 0., mn = std::numeric_limits<double>::max(), mean = 0., sd = 0.;
        for (const auto &t : trial_results) {
            const double v = tp_of(t);
            mean += v;
            mx = std::max(mx, v);
            mn = std::min(mn, v);
        }
        mean /= (double)CFG.TRIALS_NUMBER;
        for (const auto &t : trial_results) sd += std::pow(tp_of(t) - mean, 2);
        sd = std::sqrt(sd / (double)CFG.TRIALS_NUMBER);
        result.throughput_max = (size_t)mx;
        result.throughput_min = (size_t)mn;
        result.throughput_mean = (size_t)mean;
        result.throughput_std_dev = (size_t)sd;
    }
    result.iter_success_dec_alg_max = it_max;
    result.iter_success_dec_alg_min = (it_min == std::numeric_limits<size_t>::max()) ? 0 : it_min;
    result.iter_success_dec_alg_mean = it_mean;
    result.iter_success_dec_alg_std_dev = it_std;
    result.ratio_trials_success_ldpc = (double)keys / (double)CFG.TRIALS_NUMBER;
    result.ratio_trials_success_dec_alg = (double)ok / (double)CFG.TRIALS_NUMBER;
}

namespace {

// The loop's per-trial seeds (src/simulation.cpp:713-719).
std::vector<size_t> trial_seeds(size_t sim_seed, size_t count) {
    XoshiroCpp::Xoshiro256PlusPlus prng(sim_seed);
    std::uniform_int_distribution<size_t> d(0, std::numeric_limits<size_t>::max());
    std::vector<size_t> s(count);
    for (auto &x : s) x = d(prng);
    return s;
}

// run_trial for trials [0, count) of one combination from `threads` threads,
// each taking the next trial index (the reference's pool over detach_loop).
std::vector<trial_result> per_trial(const H_matrix &H, double qber, const std::vector<size_t> &seeds, size_t sim,
                                    const H_matrix_params &mp, const decoding_scaling_factors &sf, int threads) {
    std::vector<trial_result> out(seeds.size());
    std::atomic<size_t> next{0};
    std::vector<std::string> errs(threads);
    auto body = [&](int k) {
        try {
            for (size_t t; (t = next.fetch_add(1)) < seeds.size();) out[t] = run_trial(H, qber, seeds[t] + sim, mp, sf);
        } catch (const std::exception &e) {
            errs[k] = e.what();
        }
    };
    std::vector<std::thread> th;
    for (int k = 0; k < threads; ++k) th.emplace_back(body, k);
    for (auto &t : th) t.join();
    for (const auto &e : errs)
        if (!e.empty()) throw std::runtime_error(e);
    return out;
}

double secs_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void set_cfg(const char *alg, const char *max_it, size_t trials, size_t sim_seed, int threads) {
    CFG.DECODING_ALGORITHM = (size_t)std::atoi(alg);
    CFG.DECODING_ALG_MAX_ITERATIONS = (size_t)std::atoi(max_it);
    CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD = true;
    CFG.DECODING_ALG_MSG_LLR_THRESHOLD = 100.;
    CFG.TRIALS_NUMBER = trials;
    CFG.SIMULATION_SEED = sim_seed;
    CFG.THREADS_NUMBER = (size_t)threads;
    CFG.ENABLE_THROUGHPUT_MEASUREMENT = true;
}

}  // namespace

int main(int argc, char **argv) {
    try {
        const std::string mode = argc > 1 ? argv[1] : "";
        if (mode == "batch" && argc >= 12) {
            set_cfg(argv[4], argv[8], std::strtoull(argv[9], nullptr, 10), std::strtoull(argv[10], nullptr, 10),
                    std::atoi(argv[11]));
            const int threads = std::atoi(argv[11]);
            std::vector<sim_input> in(1);
            load_into(in[0].matrix, argv[2], std::atoi(argv[3]));
            in[0].matrix_path = argv[2];
            const decoding_scaling_factors sf{std::atof(argv[5]), std::atof(argv[6])};
            H_matrix_params mp;
            if (argc >= 14) {
                CFG.ENABLE_CODE_RATE_ADAPTATION = true;
                mp.punctured_bits = read_int(argv[12]);
                mp.shortened_bits = read_int(argv[13]);
            }
            std::vector<double> qbers;  // one per line, decimal text
            {
                std::ifstream f(argv[7]);
                for (double q; f >> q;) qbers.push_back(q);
            }
            for (double q : qbers) in[0].combinations.push_back({q, mp, sf});
            const auto seeds = trial_seeds(CFG.SIMULATION_SEED, CFG.TRIALS_NUMBER);
            for (size_t sim = 0; sim < qbers.size(); ++sim) {
                std::vector<trial_result> tr;
                auto t0 = std::chrono::steady_clock::now();
                qkd_ldpc_hip_run_trials(in[0].matrix, qbers[sim], seeds, sim, mp, sf, tr);
                std::printf("W seam %.6f\n", secs_since(t0));
                for (size_t t = 0; t < tr.size(); ++t)
                    std::printf("S %zu %zu %zu %d %d %lld\n", sim, t, tr[t].ldpc_res.decoding_res.iterations_num,
                                tr[t].ldpc_res.decoding_res.syndromes_match ? 1 : 0, tr[t].ldpc_res.keys_match ? 1 : 0,
                                (long long)tr[t].runtime.count());
                t0 = std::chrono::steady_clock::now();
                const auto pt = per_trial(in[0].matrix, qbers[sim], seeds, sim, mp, sf, threads);
                std::printf("W pertrial %.6f\n", secs_since(t0));
                for (size_t t = 0; t < pt.size(); ++t)
                    std::printf("T %zu %zu %zu %d %d\n", sim, t, pt[t].ldpc_res.decoding_res.iterations_num,
                                pt[t].ldpc_res.decoding_res.syndromes_match ? 1 : 0, pt[t].ldpc_res.keys_match ? 1 : 0);
            }
            for (const sim_result &r : QKD_LDPC_batch_simulation(in))
                std::printf("R %zu %.17g %.17g %zu %zu %.17g %.17g %.17g %zu %zu %zu %zu\n", r.sim_number,
                            r.ratio_trials_success_dec_alg, r.ratio_trials_success_ldpc, r.iter_success_dec_alg_max,
                            r.iter_success_dec_alg_min, r.iter_success_dec_alg_mean, r.iter_success_dec_alg_std_dev,
                            r.accurate_QBER, r.throughput_mean, r.throughput_std_dev, r.throughput_min,
                            r.throughput_max);
            return 0;
        }
        if (mode == "time" && argc >= 12) {
            set_cfg(argv[4], argv[8], std::strtoull(argv[9], nullptr, 10), std::strtoull(argv[10], nullptr, 10),
                    std::atoi(argv[11]));
            const int threads = std::atoi(argv[11]);
            H_matrix H;
            load_into(H, argv[2], std::atoi(argv[3]));
            const decoding_scaling_factors sf{std::atof(argv[5]), std::atof(argv[6])};
            const double qber = std::atof(argv[7]);
            const auto seeds = trial_seeds(CFG.SIMULATION_SEED, CFG.TRIALS_NUMBER);
            const double k = (double)(H.bit_nodes.size() - H.check_nodes.size());
            std::vector<trial_result> tr;
            // warm-up: the graph, the device workspaces and the pinned buffers
            // are built by the first call of a size (as in the reference's loop,
            // every later combination reuses them)
            // (twice: consecutive calls alternate over a device's two pipeline slots)
            qkd_ldpc_hip_run_trials(H, qber, seeds, 1, {}, sf, tr);
            qkd_ldpc_hip_run_trials(H, qber, seeds, 2, {}, sf, tr);
            auto t0 = std::chrono::steady_clock::now();
            qkd_ldpc_hip_run_trials(H, qber, seeds, 0, {}, sf, tr);
            double s = secs_since(t0);
            std::printf("seam %zu %.6f %.6g\n", seeds.size(), s, k * (double)seeds.size() / s);
            if (threads <= 0) return 0;  // (seam only)
            t0 = std::chrono::steady_clock::now();
            (void)per_trial(H, qber, seeds, 0, {}, sf, threads);
            s = secs_since(t0);
            std::printf("pertrial %zu %.6f %.6g\n", seeds.size(), s, k * (double)seeds.size() / s);
            return 0;
        }
        if (mode == "sweep" && argc >= 11) {
            set_cfg(argv[4], argv[8], std::strtoull(argv[9], nullptr, 10), std::strtoull(argv[10], nullptr, 10), 0);
            std::vector<sim_input> in(1);
            load_into(in[0].matrix, argv[2], std::atoi(argv[3]));
            in[0].matrix_path = argv[2];
            const decoding_scaling_factors sf{std::atof(argv[5]), std::atof(argv[6])};
            H_matrix_params mp;
            if (argc >= 13) {
                CFG.ENABLE_CODE_RATE_ADAPTATION = true;
                mp.punctured_bits = read_int(argv[11]);
                mp.shortened_bits = read_int(argv[12]);
            }
            std::vector<double> qbers;
            {
                std::ifstream f(argv[7]);
                for (double q; f >> q;) qbers.push_back(q);
            }
            if (qbers.empty()) throw std::runtime_error("no QBERs");
            // warm-up: two combinations build the graph, the workspaces and both
            // pipeline slots' buffers
            in[0].combinations.push_back({qbers[0], mp, sf});
            in[0].combinations.push_back({qbers[0], mp, sf});
            (void)QKD_LDPC_batch_simulation(in);
            in[0].combinations.clear();
            for (double q : qbers) in[0].combinations.push_back({q, mp, sf});
            const auto t0 = std::chrono::steady_clock::now();
            const auto res = QKD_LDPC_batch_simulation(in);
            const double s = secs_since(t0);
            double fer = 0.;
            for (const auto &r : res) fer += 1. - r.ratio_trials_success_ldpc;
            std::printf("sweep %zu %zu %.6f %.6f %.6g\n", res.size(), (size_t)CFG.TRIALS_NUMBER, s,
                        1e3 * s / (double)res.size(), fer / (double)res.size());
            return 0;
        }
        std::fprintf(stderr, "usage: batch_check batch|time|sweep ... (see the file header)\n");
        return 2;
    } catch (const std::exception &e) {
        std::printf("ERROR: %s\n", e.what());
        return 1;
    }
}
