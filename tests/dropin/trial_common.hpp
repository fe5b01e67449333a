// trial_common.hpp — helpers shared by the drop-in test drivers
// (run_trial_check.cpp, batch_check.cpp): the reference's trial generator
// (fill_random_bits / inject_errors, src/array_and_matrix_operations.cpp:
// 889-933), a matrix loader into its H_matrix through the C ABI, and list
// files.  Test infrastructure.
#pragma once

#include <algorithm>
#include <fstream>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "qkd_ldpc_algorithm.hpp"  // tests/dropin/api: the reference's interface
#include "qkd_ldpc_hip.h"

namespace trial_common {

// fill_random_bits / inject_errors (src/array_and_matrix_operations.cpp:889-933).
inline void fill_random_bits(XoshiroCpp::Xoshiro256PlusPlus &prng, std::vector<int> &bit_array) {
    std::uniform_int_distribution<int> distribution(0, 1);
    for (size_t i = 0; i < bit_array.size(); ++i) bit_array[i] = distribution(prng);
}

inline double inject_errors(XoshiroCpp::Xoshiro256PlusPlus &prng, const std::vector<int> &bit_array, double QBER,
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

inline void load_into(H_matrix &H, const char *path, int fmt) {
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

inline std::vector<unsigned long long> read_u64(const char *path) {
    std::ifstream in(path);
    if (!in) throw std::runtime_error(std::string("cannot open ") + path);
    std::vector<unsigned long long> v;
    unsigned long long x;
    while (in >> x) v.push_back(x);
    return v;
}

inline std::vector<int> read_int(const char *path) {
    std::vector<int> v;
    for (unsigned long long x : read_u64(path)) v.push_back((int)x);
    return v;
}

}  // namespace trial_common
