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
//   run_trial_check reuse  <matrixA> <fmtA> <matrixB> <fmtB> <alg> <primary> <secondary> <qber> <max_it> <seeds.txt>
//       the reference's config-after-config loop: trials on A, then B loaded
//       INTO THE SAME H_matrix object (same address, same n/m/nnz when B is a
//       column permutation of A), trials on B: "A ..." / "B ..." lines.
// Failures print "ERROR: <what>" and exit 1, like the reference's main.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "qkd_ldpc_algorithm.hpp"  // tests/dropin/api: the reference's interface
#include "qkd_ldpc_hip.h"

config_data CFG;  // defined by the reference's src/config.cpp

namespace {

// fill_random_bits / inject_errors (src/array_and_matrix_operations.cpp:889-933).
void fill_random_bits(XoshiroCpp::Xoshiro256PlusPlus &prng, std::vector<int> &bit_array) {
    std::uniform_int_distribution<int> distribution(0, 1);
    for (size_t i = 0; i < bit_array.size(); ++i) bit_array[i] = distribution(prng);
}

double inject_errors(XoshiroCpp::Xoshiro256PlusPlus &prng, const std::vector<int> &bit_array, double QBER,
                     std::vector<int> &out) {
    const size_t len = bit_array.size();
    const size_t num_errors = static_cast<size_t>(static_cast<double>(len) * QBER);
    out = bit_array;
    if (num_errors > 0) {
        std::vector<size_t> pos(len);
        for (size_t i = 0; i < len; ++i) pos[i] = i;
        std::shuffle(pos.begin(), pos.end(), prng);
        for (size_t i = 0; i < num_errors; ++i) out[pos[i]] ^= 1;
    }
    return static_cast<double>(num_errors) / static_cast<double>(len);
}

void load_into(H_matrix &H, const char *path, int fmt) {
    int32_t n = 0, m = 0, nnz = 0, reg = 0;
    if (qldpc_load_matrix(path, fmt, &n, &m, &nnz, nullptr, nullptr, nullptr, nullptr, &reg))
        throw std::runtime_error(qldpc_last_error());
    std::vector<int32_t> rp(m + 1), ci(nnz), cp(n + 1), ri(nnz);
    if (qldpc_load_matrix(path, fmt, &n, &m, &nnz, rp.data(), ci.data(), cp.data(), ri.data(), &reg))
        throw std::runtime_error(qldpc_last_error());
    H.check_nodes.assign(m, {});
    for (int j = 0; j < m; ++j) H.check_nodes[j].assign(ci.begin() + rp[j], ci.begin() + rp[j + 1]);
    H.bit_nodes.assign(n, {});
    for (int i = 0; i < n; ++i) H.bit_nodes[i].assign(ri.begin() + cp[i], ri.begin() + cp[i + 1]);
    H.is_regular = reg != 0;
}

std::vector<unsigned long long> read_u64(const char *path) {
    std::ifstream in(path);
    if (!in) throw std::runtime_error(std::string("cannot open ") + path);
    std::vector<unsigned long long> v;
    unsigned long long x;
    while (in >> x) v.push_back(x);
    return v;
}

std::vector<int> read_int(const char *path) {
    std::vector<int> v;
    for (unsigned long long x : read_u64(path)) v.push_back((int)x);
    return v;
}

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
        std::fprintf(stderr, "usage: run_trial_check load|trials|reuse ... (see the file header)\n");
        return 2;
    } catch (const std::exception &e) {
        std::printf("ERROR: %s\n", e.what());
        return 1;
    }
}
