// host_mirror_check — exercises the C++ mirror (qkd_ldpc_algorithm.hpp) the
// way the reference's example program does (example/qkd_ldpc_example.cpp).
//   host_mirror_check load <matrix> <format>   parse only (no GPU): "n m nnz regular"
//   host_mirror_check kat <matrix>             Johnson Ex. 2.5 through QKD_LDPC (GPU)
//   host_mirror_check decoders <matrix> <format> <frames.bin> <out.bin>   (GPU)
//       frames.bin: int32 batch, then per frame n doubles (llr) + m int32 (syndrome).
//       Factors: NMSA 0.78, OMSA 0.77, ANMSA 0.8/0.35, AOMSA 0.55/1.2; 50 its, thr 100.
//       Runs each of the six per-frame decoders on every frame, and decode_batch
//       for all frames, checks the two agree, and writes per algorithm and frame
//       iterations (u32), syndromes_match (u8) and bits (n x u8) to out.bin.
// Failures print "ERROR: <what>" and exit 1, like the reference's main.
#include <cstdio>
#include <cstdlib>
#include <fstream>
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
        if (argc >= 6 && std::string(argv[1]) == "decoders") {
            const int fmt = std::atoi(argv[3]);
            H_matrix H = fmt == 0   ? read_sparse_uncompressed_matrix(argv[2])
                         : fmt == 1 ? read_sparse_matrix_alist(argv[2])
                         : fmt == 2 ? read_sparse_matrix_1(argv[2])
                                    : read_sparse_matrix_2(argv[2]);
            const size_t n = H.bit_nodes.size(), m = H.check_nodes.size();
            std::ifstream in(argv[4], std::ios::binary);
            int32_t batch = 0;
            in.read(reinterpret_cast<char *>(&batch), 4);
            double fac[6][2] = {{0, 0}, {0, 0}, {0.78, 0}, {0.77, 0}, {0.8, 0.35}, {0.55, 1.2}};
            std::vector<std::vector<double>> llr(batch, std::vector<double>(n));
            std::vector<std::vector<int>> synd(batch, std::vector<int>(m));
            for (int f = 0; f < batch; ++f) {
                in.read(reinterpret_cast<char *>(llr[f].data()), n * 8);
                in.read(reinterpret_cast<char *>(synd[f].data()), m * 4);
            }
            if (!in) throw std::runtime_error("frames file truncated");
            CFG.DECODING_ALG_MAX_ITERATIONS = 50;
            CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD = true;
            CFG.DECODING_ALG_MSG_LLR_THRESHOLD = 100.;
            std::ofstream out(argv[5], std::ios::binary);
            for (int alg = 0; alg < 6; ++alg) {
                std::vector<double> flat(batch * n);
                std::vector<uint8_t> fs(batch * m), bb;
                for (int f = 0; f < batch; ++f) {
                    std::copy(llr[f].begin(), llr[f].end(), flat.begin() + f * n);
                    for (size_t j = 0; j < m; ++j) fs[f * m + j] = (uint8_t)synd[f][j];
                }
                CFG.DECODING_ALGORITHM = alg;
                const decoding_scaling_factors sf{fac[alg][0], fac[alg][1]};
                const auto res = decode_batch(H, flat, fs, batch, sf, bb);
                for (int f = 0; f < batch; ++f) {
                    std::vector<int> bits(n);
                    const size_t it = 50;
                    const double thr = 100.;
                    decoding_result r;
                    switch (alg) {
                    case 0: r = sum_product_decoding(llr[f], H, synd[f], it, thr, bits); break;
                    case 1: r = sum_product_linear_approx_decoding(llr[f], H, synd[f], it, thr, bits); break;
                    case 2: r = min_sum_normalized_decoding(llr[f], H, synd[f], it, sf.primary, thr, bits); break;
                    case 3: r = min_sum_offset_decoding(llr[f], H, synd[f], it, sf.primary, thr, bits); break;
                    case 4:
                        r = adaptive_min_sum_normalized_decoding(llr[f], H, synd[f], it, sf.primary, sf.secondary, thr,
                                                                 bits);
                        break;
                    default:
                        r = adaptive_min_sum_offset_decoding(llr[f], H, synd[f], it, sf.primary, sf.secondary, thr,
                                                             bits);
                    }
                    if (r.iterations_num != res[f].iterations_num || r.syndromes_match != res[f].syndromes_match)
                        throw std::runtime_error("per-frame decoder and decode_batch disagree (results)");
                    for (size_t i = 0; i < n; ++i)
                        if ((uint8_t)bits[i] != bb[f * n + i])
                            throw std::runtime_error("per-frame decoder and decode_batch disagree (bits)");
                    const uint32_t it32 = (uint32_t)r.iterations_num;
                    const uint8_t ok = r.syndromes_match ? 1 : 0;
                    out.write(reinterpret_cast<const char *>(&it32), 4);
                    out.write(reinterpret_cast<const char *>(&ok), 1);
                    out.write(reinterpret_cast<const char *>(&bb[f * n]), n);
                }
            }
            std::printf("OK %d frames x 6 decoders\n", batch);
            return 0;
        }
        std::fprintf(stderr, "usage: host_mirror_check load <matrix> <format> | kat <matrix> | decoders ...\n");
        return 2;
    } catch (const std::exception &e) {
        std::printf("ERROR: %s\n", e.what());
        return 1;
    }
}
