// run_trial_check — the reference's run_trial (src/simulation.cpp:540-576),
// restated over the drop-in replacement TU (qkd_ldpc_v_amd/host/dropin/
// qkd_ldpc_algorithm.cpp) compiled against the reference-shaped declarations
// in tests/dropin/api/.  Test infrastructure (tests/test_dropin.py).
//
//   run_trial_check load   <matrix> <format>
//       parse only (no GPU): "n m nnz"
//   run_trial_check trials <matrix> <format> <alg> <primary> <secondary> <qber> <max_it> <seeds.txt>
//                          [<punctured.txt> <shortened.txt>]
//       per seed: XoshiroCpp::Xoshiro256PlusPlus prng(seed); Alice =
//       fill_random_bits, Bob = inject_errors (src/array_and_matrix_operations.cpp:
//       889-933); then exactly run_trial's call — QKD_LDPC_RATE_ADAPT(matrix,
//       alice, bob, q, sf, params, prng) when position lists are given
//       (CFG.ENABLE_CODE_RATE_ADAPTATION), else QKD_LDPC(matrix, alice, bob, q,
//       sf, params).  Prints "iterations syndromes_match keys_match" per trial.
//   run_trial_check badsyndrome <matrix> <format>
//       sum_product_decoding with a syndrome holding a 2 (no GPU needed: the
//       drop-in refuses it before any device work) -> "ERROR: ..."
//   run_trial_check keycost <matrix> <format> <reps>
//       host cost of the graph cache's keys per decoder call (no GPU):
//       "keycost_us fast <us> full <us>" — the O(1) key every call takes, the
//       full content fingerprint a miss takes
//   run_trial_check reuse  <matrixA> <fmtA> <matrixB> <fmtB> <alg> <primary> <secondary> <qber> <max_it> <seeds.txt>
//       the reference's config-after-config loop: trials on A, then B loaded
//       INTO THE SAME H_matrix object (same address, same n/m/nnz when B is a
//       column permutation of A), trials on B: "A ..." / "B ..." lines.
//   run_trial_check inplace <matrix> <format>
//       the graph cache after an in-place edit its O(1) key cannot see (two
//       unsampled rows swap their check ids): "inplace fastkey_same 1
//       detected_after <calls>" — the periodic full check's catch.
// Failures print "ERROR: <what>" and exit 1, like the reference's main.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "qkd_ldpc_algorithm.hpp"  // tests/dropin/api: the reference's interface
#include "qkd_ldpc_hip.h"
#include "trial_common.hpp"
#include "../../qkd_ldpc_v_amd/host/qkd_ldpc_impl.hpp"
#include <chrono>

config_data CFG;  // defined by the reference's src/config.cpp

namespace {

using namespace trial_common;

struct trial_result {  // src/simulation.hpp: the fields run_trial fills
    LDPC_result ldpc_res{};
    double accurate_QBER{};
};

// run_trial (src/simulation.cpp:540-576) minus the throughput timer.
trial_result run_trial(const H_matrix &matrix, double QBER, size_t seed, const H_matrix_params &matrix_params,
                       const decoding_scaling_factors &scaling_factors) {
    trial_result result;
    XoshiroCpp::Xoshiro256PlusPlus prng(seed);
    const size_t num_bit_nodes = matrix.bit_nodes.size();
    std::vector<int> alice_bit_array(num_bit_nodes);
    std::vector<int> bob_bit_array(num_bit_nodes);
    fill_random_bits(prng, alice_bit_array);
    result.accurate_QBER = inject_errors(prng, alice_bit_array, QBER, bob_bit_array);
    if (result.accurate_QBER == 0.)
        throw std::runtime_error("Key size '" + std::to_string(num_bit_nodes) + "' is too small for QBER.");
    if (CFG.ENABLE_CODE_RATE_ADAPTATION)
        result.ldpc_res = QKD_LDPC_RATE_ADAPT(matrix, alice_bit_array, bob_bit_array, result.accurate_QBER,
                                              scaling_factors, matrix_params, prng);
    else
        result.ldpc_res = QKD_LDPC(matrix, alice_bit_array, bob_bit_array, result.accurate_QBER, scaling_factors,
                                   matrix_params);
    return result;
}

void print(const char *tag, const trial_result &r) {
    std::printf("%s%zu %d %d\n", tag, r.ldpc_res.decoding_res.iterations_num,
                r.ldpc_res.decoding_res.syndromes_match ? 1 : 0, r.ldpc_res.keys_match ? 1 : 0);
}

void set_cfg(const char *alg, const char *max_it) {
    CFG.DECODING_ALGORITHM = (size_t)std::atoi(alg);
    CFG.DECODING_ALG_MAX_ITERATIONS = (size_t)std::atoi(max_it);
    CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD = true;
    CFG.DECODING_ALG_MSG_LLR_THRESHOLD = 100.;
}

}  // namespace

int main(int argc, char **argv) {
    try {
        const std::string mode = argc > 1 ? argv[1] : "";
        if (mode == "load" && argc >= 4) {
            H_matrix H;
            load_into(H, argv[2], std::atoi(argv[3]));
            size_t nnz = 0;
            for (const auto &r : H.check_nodes) nnz += r.size();
            std::printf("%zu %zu %zu\n", H.bit_nodes.size(), H.check_nodes.size(), nnz);
            return 0;
        }
        if (mode == "badsyndrome" && argc >= 4) {
            H_matrix H;
            load_into(H, argv[2], std::atoi(argv[3]));
            set_cfg("0", "50");
            std::vector<double> llr(H.bit_nodes.size(), 3.0);
            std::vector<int> synd(H.check_nodes.size(), 0), out(H.bit_nodes.size());
            synd[1] = 2;
            (void)sum_product_decoding(llr, H, synd, 50, 100.0, out);
            std::printf("accepted\n");
            return 0;
        }
        if (mode == "keycost" && argc >= 5) {
            H_matrix H;
            load_into(H, argv[2], std::atoi(argv[3]));
            const int reps = std::atoi(argv[4]);
            uint64_t sink = 0;
            const auto t0 = std::chrono::steady_clock::now();
            for (int r = 0; r < reps; ++r) sink ^= qkd_ldpc_v_amd::impl::fast_key_of(H).sample;
            const double fast = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            const auto t1 = std::chrono::steady_clock::now();
            for (int r = 0; r < reps; ++r) sink ^= qkd_ldpc_v_amd::impl::key_of(H).h;
            const double full = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count();
            std::printf("keycost_us fast %.3f full %.3f %llu\n", fast / reps, full / reps, (unsigned long long)(sink & 1));
            return 0;
        }
        if (mode == "trials" && argc >= 10) {
            H_matrix H;
            load_into(H, argv[2], std::atoi(argv[3]));
            set_cfg(argv[4], argv[8]);
            const decoding_scaling_factors sf{std::atof(argv[5]), std::atof(argv[6])};
            const double qber = std::atof(argv[7]);
            H_matrix_params mp;
            if (argc >= 12) {
                CFG.ENABLE_CODE_RATE_ADAPTATION = true;
                mp.punctured_bits = read_int(argv[10]);
                mp.shortened_bits = read_int(argv[11]);
            }
            for (unsigned long long seed : read_u64(argv[9])) print("", run_trial(H, qber, (size_t)seed, mp, sf));
            return 0;
        }
        if (mode == "reuse" && argc >= 12) {
            H_matrix H;  // one object for both configurations, as the reference's loop
            set_cfg(argv[6], argv[10]);
            const decoding_scaling_factors sf{std::atof(argv[7]), std::atof(argv[8])};
            const double qber = std::atof(argv[9]);
            const auto seeds = read_u64(argv[11]);
            load_into(H, argv[2], std::atoi(argv[3]));
            for (unsigned long long seed : seeds) print("A ", run_trial(H, qber, (size_t)seed, {}, sf));
            load_into(H, argv[4], std::atoi(argv[5]));
            for (unsigned long long seed : seeds) print("B ", run_trial(H, qber, (size_t)seed, {}, sf));
            return 0;
        }
        if (mode == "inplace" && argc >= 4) {
            // an in-place edit of H that the O(1) fast key cannot see: two rows
            // and the bits they hold, none of them among the 128 sampled lists,
            // swap their check ids; the cache must pick up the new content by
            // its periodic full check
            H_matrix H;
            load_into(H, argv[2], std::atoi(argv[3]));
            namespace qi = qkd_ldpc_v_amd::impl;
            auto &cache = qi::graph_cache();
            const auto e0 = cache.get(H);
            const size_t m = H.check_nodes.size(), n = H.bit_nodes.size();
            const size_t rs = m > 64 ? m / 64 : 1, cs = n > 64 ? n / 64 : 1;
            auto free_row = [&](size_t j) {
                if (j % rs == 0) return false;
                for (int b : H.check_nodes[j])
                    if ((size_t)b % cs == 0) return false;
                return true;
            };
            size_t j1 = m, j2 = m;
            for (size_t j = 0; j < m && j2 == m; ++j)
                if (free_row(j)) (j1 == m ? j1 : j2) = j;
            if (j2 == m) throw std::runtime_error("no pair of unsampled rows");
            const auto fk0 = qi::fast_key_of(H);
            std::swap(H.check_nodes[j1], H.check_nodes[j2]);  // (swaps the buffers: unsampled rows)
            for (size_t j : {j1, j2})
                for (int b : H.check_nodes[j]) {
                    auto &col = H.bit_nodes[b];
                    for (int &x : col) x = (x == (int)j1) ? (int)j2 : (x == (int)j2) ? (int)j1 : x;
                    std::sort(col.begin(), col.end());
                }
            const bool same = qi::fast_key_of(H) == fk0;
            int detected = -1;
            for (int c = 1; c <= 64 && detected < 0; ++c)
                if (cache.get(H) != e0) detected = c;
            std::printf("inplace fastkey_same %d detected_after %d\n", same ? 1 : 0, detected);
            return 0;
        }
        std::fprintf(stderr, "usage: run_trial_check load|trials|reuse|inplace ... (see the file header)\n");
        return 2;
    } catch (const std::exception &e) {
        std::printf("ERROR: %s\n", e.what());
        return 1;
    }
}
