// loaders.hpp — H-matrix adjacency as the reference holds it
// (H_matrix, ColdCloudd/QKD_LDPC_V src/array_and_matrix_operations.hpp:60-77).
#pragma once
#include <stdexcept>
#include <string>
#include <vector>

namespace qldpc {

struct LoadError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

struct HMatrix {
    std::vector<std::vector<int>> bit_nodes;    // per bit: its check ids (file order)
    std::vector<std::vector<int>> check_nodes;  // per check: its bit ids (file order)
    bool is_regular = false;
};

// format: 0 uncompressed, 1 alist, 2 sparse_1, 3 sparse_2 (reference src/config.hpp:202).
HMatrix load_matrix(const std::string &path, int format);

}  // namespace qldpc
