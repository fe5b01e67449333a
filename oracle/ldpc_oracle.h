/* ldpc_oracle.h — CPU ORACLE for the QKD-LDPC decode hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is a plain-C restatement of the reference
 * decoders (ColdCloudd/QKD_LDPC_V src/qkd_ldpc_algorithm.cpp:3-1029) and of the
 * per-trial frame construction (QKD_LDPC, :1031-1119), written from the
 * reference's semantics.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path (qkd_ldpc_v_amd, the HIP
 * library) never links or calls it.
 *
 * Parity pinning: the reference has no tests; its only known-answer case is
 * example/qkd_ldpc_example.cpp (Johnson Ex. 2.5).  tests/golden/kat_johnson.json
 * holds that KAT's outputs as recorded from the reference (SURVEY.md §3(5),
 * §8c).  The reference itself cannot be compiled here (its headers need
 * XoshiroCpp.hpp and CPM-fetched packages absent from this image), so the
 * oracle is pinned by that KAT plus the glibc bit-exactness of the math it
 * calls.  See DESIGN.md §Oracle.
 */
#ifndef QKD_LDPC_ORACLE_H
#define QKD_LDPC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Decoder ids — reference src/config.hpp:201 (DEC_SPA .. DEC_AOMSA). */
enum { QLO_SPA = 0, QLO_SPA_LIN = 1, QLO_NMSA = 2, QLO_OMSA = 3, QLO_ANMSA = 4, QLO_AOMSA = 5 };

typedef struct qlo_graph qlo_graph;

/* Build from the reference's two adjacency lists, flattened:
 *   check_nodes (H_matrix::check_nodes, src/array_and_matrix_operations.hpp:68)
 *       -> rowptr[m+1], colidx[E]   (row j lists its bit ids in file order)
 *   bit_nodes   (H_matrix::bit_nodes, :64)
 *       -> colptr[n+1], rowidx[E]   (bit i lists its check ids in file order)
 * The lists need not be sorted: the oracle reproduces the reference's
 * occurrence-counter slot pairing (check_pos_idx / bit_pos_idx,
 * src/qkd_ldpc_algorithm.cpp:67-69,116-118).  Returns NULL if the two lists do
 * not describe the same number of edges per bit / per check. */
qlo_graph *qlo_graph_new(int32_t n, int32_t m, const int32_t *rowptr, const int32_t *colidx,
                         const int32_t *colptr, const int32_t *rowidx);
void qlo_graph_free(qlo_graph *g);

/* s[j] = XOR of bits[check_nodes[j][k]] — calculate_syndrome,
 * src/array_and_matrix_operations.cpp:936-950. */
void qlo_syndrome(const qlo_graph *g, const uint8_t *bits, uint8_t *synd);

typedef struct {
    int32_t alg;            /* QLO_* */
    int32_t max_iterations; /* DECODING_ALG_MAX_ITERATIONS */
    int32_t thr_enabled;    /* ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD */
    double thr;             /* DECODING_ALG_MSG_LLR_THRESHOLD */
    double primary;         /* alpha (NMSA/ANMSA) or beta (OMSA/AOMSA) */
    double secondary;       /* nu (ANMSA) or sigma (AOMSA) */
} qlo_params;

/* One frame.  Mirrors the six decoders' contract: llr[n] a-priori LLRs,
 * synd[m] target syndrome, out[n] decoded hard bits (the reference's
 * bit_array_out).  post[n] (nullable) receives the reference's total_bit_llr at
 * return.  Returns iterations_num; *synd_ok = syndromes_match. */
int32_t qlo_decode(const qlo_graph *g, const qlo_params *p, const double *llr, const uint8_t *synd,
                   uint8_t *out, double *post, int32_t *synd_ok);

/* Per-iteration trace hook (the reference's TRACE_DECODING_ALG prints of L, z,
 * s — src/qkd_ldpc_algorithm.cpp:88-99).  trace_post[it*n + i] = total_bit_llr
 * after iteration it (for it < returned iterations, where computed). */
int32_t qlo_decode_trace(const qlo_graph *g, const qlo_params *p, const double *llr,
                         const uint8_t *synd, uint8_t *out, double *post, int32_t *synd_ok,
                         double *trace_post);

/* Batch of independent frames on `threads` host threads (one frame per task,
 * the reference's BS::thread_pool model, src/simulation.cpp:721,740-746). */
void qlo_decode_batch(const qlo_graph *g, const qlo_params *p, int32_t batch, const double *llr,
                      const uint8_t *synd, uint8_t *out, uint32_t *iters, uint8_t *synd_ok,
                      double *post, int32_t threads);

/* QKD_LDPC frame construction (src/qkd_ldpc_algorithm.cpp:1043-1052):
 * log_p = log((1-q)/q); llr[i] = bob[i] ? -log_p : log_p; synd = H*alice. */
void qlo_build_frame(const qlo_graph *g, const uint8_t *alice, const uint8_t *bob, double qber,
                     double *llr, uint8_t *synd);

/* Full per-trial entry QKD_LDPC (without privacy maintenance output):
 * frame construction + decode + keys_match (src/qkd_ldpc_algorithm.cpp:1031-1087). */
int32_t qlo_qkd_ldpc(const qlo_graph *g, const qlo_params *p, const uint8_t *alice,
                     const uint8_t *bob, double qber, uint8_t *bob_solution,
                     int32_t *synd_ok, int32_t *keys_match);

#ifdef __cplusplus
}
#endif
#endif
