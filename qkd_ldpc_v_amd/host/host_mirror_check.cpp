// host_mirror_check — exercises the C++ mirror (qkd_ldpc_algorithm.hpp) the
// way the reference's example program does (example/qkd_ldpc_example.cpp).
//   host_mirror_check load <matrix> <format>   parse only (no GPU): "n m nnz regular"
//   host_mirror_check kat <matrix>             Johnson Ex. 2.5 through QKD_LDPC (GPU)
// Failures print "ERROR: <what>" and exit 1, like the reference's main.
#include <cstdio>
#include <cstdlib>
#include <string>

#include "../host/qkd_ldpc_algorithm.hpp"

using namespace qkd_ldpc_v_amd;

int main(int argc, char **argv) {
    try {
        if (argc >= 4 && std::string(argv[1]) == "load") {
            const int fmt = std::atoi(argv[3]);
            H_matrix H = fmt == 0   ? read_sparse_uncompressed_matrix(argv[2])
                         : fmt == 1 ? read_sparse_matrix_alist(argv[2])
                         : fmt == 2 ? read_sparse_matrix_1(argv[2])
                                    : read_sparse_matrix_2(argv[2]);
            size_t nnz = 0;
            for (const auto &r : H.check_nodes) nnz += r.size();
            std::printf("%zu %zu %zu %d\n", H.bit_nodes.size(), H.check_nodes.size(), nnz, H.is_regular ? 1 : 0);
            return 0;
        }
        if (argc >= 3 && std::string(argv[1]) == "kat") {
            CFG.DECODING_ALG_MAX_ITERATIONS = 100;
            CFG.DECODING_ALGORITHM = DEC_SPA;
            CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD = true;
            CFG.DECODING_ALG_MSG_LLR_THRESHOLD = 100.;
            H_matrix matrix = read_sparse_uncompressed_matrix(argv[2]);
            std::vector<int> alice{0, 0, 1, 0, 1, 1};
            std::vector<int> bob{1, 0, 1, 0, 1, 1};
            LDPC_result r = QKD_LDPC(matrix, alice, bob, 0.2);
            std::printf("iterations=%zu syndromes_match=%d keys_match=%d\n", r.decoding_res.iterations_num,
                        r.decoding_res.syndromes_match ? 1 : 0, r.keys_match ? 1 : 0);
            return 0;
        }
        std::fprintf(stderr, "usage: host_mirror_check load <matrix> <format> | kat <matrix>\n");
        return 2;
    } catch (const std::exception &e) {
        std::printf("ERROR: %s\n", e.what());
        return 1;
    }
}
