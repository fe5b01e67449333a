/* qkd_ldpc_hip.h — C ABI of libqkdldpc_hip.so, the MI355X (gfx950) LDPC
 * belief-propagation decoder for QKD error reconciliation.
 *
 * This is the drop-in boundary for the hot path of ColdCloudd/QKD_LDPC_V:
 * the six flooding decoders of src/qkd_ldpc_algorithm.cpp:3-1029 (declared at
 * src/qkd_ldpc_algorithm.hpp:28-90), batched over independent trials — the
 * pool.detach_loop seam at src/simulation.cpp:740-746 — plus the per-trial frame
 * construction of QKD_LDPC (src/qkd_ldpc_algorithm.cpp:1031-1087) and the H
 * loaders it reads (src/array_and_matrix_operations.cpp:291-886).
 *
 * Plain C: pointers and sizes only.  Every entry returns 0 on success and a
 * negative QLDPC_E* code on failure; qldpc_last_error() then describes it
 * (thread-local).  The C++ mirror in qkd_ldpc_v_amd/host/qkd_ldpc_algorithm.hpp
 * turns failures into std::runtime_error, as the reference's loaders do.
 */
#ifndef QKD_LDPC_HIP_H
#define QKD_LDPC_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QLDPC_OK 0
#define QLDPC_EINVAL (-1)   /* bad argument / malformed graph */
#define QLDPC_EHIP (-2)     /* HIP runtime failure */
#define QLDPC_EIO (-3)      /* matrix file cannot be opened / parsed */
#define QLDPC_ENOMEM (-4)
#define QLDPC_EUNSUP (-5)   /* graph shape the GPU path does not accept */

/* Decoder ids: reference src/config.hpp:201 (DEC_SPA=0 ... DEC_AOMSA=5). */
#define QLDPC_SPA 0
#define QLDPC_SPA_LIN 1
#define QLDPC_NMSA 2
#define QLDPC_OMSA 3
#define QLDPC_ANMSA 4
#define QLDPC_AOMSA 5

/* Matrix file formats: reference src/config.hpp:202 (MAT_*). */
#define QLDPC_MAT_UNCOMPRESSED 0
#define QLDPC_MAT_ALIST 1
#define QLDPC_MAT_SPARSE_1 2
#define QLDPC_MAT_SPARSE_2 3

typedef struct qldpc_graph qldpc_graph;

/* Decoder parameters.  Replaces the per-call arguments of the six decoders
 * (src/qkd_ldpc_algorithm.hpp:28-90) plus the global-CFG inputs they read:
 * CFG.DECODING_ALGORITHM (dispatch at src/qkd_ldpc_algorithm.cpp:1056-1085),
 * CFG.DECODING_ALG_MAX_ITERATIONS, CFG.ENABLE_DECODING_ALG_MSG_LLR_THRESHOLD and
 * CFG.DECODING_ALG_MSG_LLR_THRESHOLD; primary/secondary are
 * decoding_scaling_factors (src/config.hpp:50-54). */
typedef struct {
    int32_t algorithm;      /* QLDPC_SPA .. QLDPC_AOMSA */
    int32_t max_iterations; /* >= 1 */
    int32_t thr_enabled;    /* message LLR clipping on/off */
    int32_t reserved;
    double thr;             /* clipping threshold (> 0 when enabled) */
    double primary;         /* alpha (NMSA, ANMSA) or beta (OMSA, AOMSA) */
    double secondary;       /* nu (ANMSA) or sigma (AOMSA) */
} qldpc_params;

/* ---------------------------------------------------------------- loaders */

/* Parse a parity-check matrix file into the reference's H_matrix adjacency
 * (check_nodes -> row_ptr/col_idx, bit_nodes -> col_ptr/row_idx).  Restates
 * read_sparse_uncompressed_matrix / read_sparse_matrix_alist /
 * read_sparse_matrix_1 / read_sparse_matrix_2
 * (src/array_and_matrix_operations.cpp:764-886, 291-468, 478-617, 626-761),
 * including their validation errors.  Files ending in ".gz" are inflated first.
 * Call with NULL arrays to query n, m and nnz; then again with buffers of
 * m+1, nnz, n+1 and nnz entries.  *is_regular mirrors H_matrix::is_regular. */
int qldpc_load_matrix(const char *path, int32_t format, int32_t *n, int32_t *m, int32_t *nnz,
                      int32_t *row_ptr, int32_t *col_idx, int32_t *col_ptr, int32_t *row_idx,
                      int32_t *is_regular);

/* ------------------------------------------------------------------ graph */

/* Build the device-resident Tanner graph from check_nodes in CSR form
 * (row_ptr[m+1], col_idx[nnz]), bit_nodes taken as their ascending transpose.
 * The graph is immutable, replicated on every device of device_mask (bit d =
 * HIP device d; 0 = current device only) and safe to share between host
 * threads.  Rows out of ascending order decode with the reference's occurrence
 * pairing (see qldpc_graph_create_checked); a bit listed twice in one row
 * returns QLDPC_EUNSUP. */
int qldpc_graph_create(int32_t n, int32_t m, const int32_t *row_ptr, const int32_t *col_idx,
                       int32_t device_mask, qldpc_graph **out);

/* As qldpc_graph_create with the caller's bit_nodes (col_ptr[n+1],
 * row_idx[nnz], the reference's H_matrix::bit_nodes in its own order).  When
 * check_nodes rows are ascending and bit_nodes is their ascending transpose,
 * the reference's slot counters (src/qkd_ldpc_algorithm.cpp:67-69,116-118) pair
 * every message with its own edge; otherwise they pair an edge's b2c with
 * another edge's message, and the graph decodes with that occurrence pairing
 * (the v1 global-slot kernel and a pairing pass).  Lists that disagree on an
 * edge count return QLDPC_EUNSUP. */
int qldpc_graph_create_checked(int32_t n, int32_t m, const int32_t *row_ptr,
                               const int32_t *col_idx, const int32_t *col_ptr,
                               const int32_t *row_idx, int32_t device_mask, qldpc_graph **out);

/* As qldpc_graph_create, on an explicit list of HIP devices, one shard per
 * entry: qldpc_decode_batch splits a batch in ndevices contiguous slices, one
 * host thread, stream and graph replica per entry.  A device may be listed
 * more than once (several concurrent shards on one GPU). */
int qldpc_graph_create_on(int32_t n, int32_t m, const int32_t *row_ptr, const int32_t *col_idx,
                          const int32_t *devices, int32_t ndevices, qldpc_graph **out);

/* qldpc_graph_create_checked on an explicit device list (one shard per entry,
 * as qldpc_graph_create_on): the C++ drop-in's graphs (the node's GPUs, or
 * logical shards of one GPU for tests). */
int qldpc_graph_create_checked_on(int32_t n, int32_t m, const int32_t *row_ptr, const int32_t *col_idx,
                                  const int32_t *col_ptr, const int32_t *row_idx, const int32_t *devices,
                                  int32_t ndevices, qldpc_graph **out);

/* Plan only, on the host (no device is touched): the returned graph has no
 * devices and cannot decode; it answers qldpc_graph_info and
 * qldpc_graph_labels.  For inspection and CPU tests of the planner. */
int qldpc_graph_create_host(int32_t n, int32_t m, const int32_t *row_ptr, const int32_t *col_idx,
                            qldpc_graph **out);

void qldpc_graph_destroy(qldpc_graph *g);

/* n, m, nnz and the number of devices the graph lives on. */
int qldpc_graph_info(const qldpc_graph *g, int32_t *n, int32_t *m, int32_t *nnz,
                     int32_t *num_devices);

/* ----------------------------------------------------------------- decode */

/* Decode `batch` independent frames held in HOST memory; synchronous.
 * Replaces `batch` calls of the decoder selected by p->algorithm, each
 *   decoding_result f(llr, H, syndrome, max_it, [alpha|beta], [nu|sigma], thr, out)
 * (src/qkd_ldpc_algorithm.hpp:28-90).  llr: batch*n doubles (frame-major),
 * syndrome: batch*m bytes in {0,1}, bits_out: batch*n bytes (bit_array_out),
 * iters_out / synd_ok_out: decoding_result {iterations_num, syndromes_match}
 * per frame, posterior_out (nullable): batch*n doubles = the reference's
 * total_bit_llr at return.  Frames are split in contiguous slices over the
 * graph's devices, one host thread per device, no collectives. */
int qldpc_decode_batch(qldpc_graph *g, const qldpc_params *p, int32_t batch, const double *llr,
                       const uint8_t *syndrome, uint8_t *bits_out, uint32_t *iters_out,
                       uint8_t *synd_ok_out, double *posterior_out);

/* Same on DEVICE buffers of the graph's device `device`, enqueued on the HIP
 * stream `stream` (hipStream_t; NULL = default stream).  Asynchronous. */
int qldpc_decode_batch_device(qldpc_graph *g, int32_t device, const qldpc_params *p, int32_t batch,
                              const double *d_llr, const uint8_t *d_syndrome, uint8_t *d_bits_out,
                              uint32_t *d_iters_out, uint8_t *d_synd_ok_out,
                              double *d_posterior_out, void *stream);

/* ------------------------------------------------ per-trial frame (QKD_LDPC) */

/* QKD_LDPC's frame construction on device (src/qkd_ldpc_algorithm.cpp:
 * 1043-1052): llr[i] = bob[i] ? -log_p : log_p, syndrome = H * alice
 * (calculate_syndrome, src/array_and_matrix_operations.cpp:936-950).
 * d_alice/d_bob: batch*n bytes in {0,1}.  d_log_p: batch doubles, each
 * log((1-q)/q) of the trial's accurate QBER q evaluated by the HOST C library
 * (qldpc_log_p below): glibc's log is not correctly rounded, so evaluating it
 * anywhere else could move an LLR by an ulp. */
int qldpc_build_frames_device(qldpc_graph *g, int32_t device, int32_t batch, const uint8_t *d_alice,
                              const uint8_t *d_bob, const double *d_log_p, double *d_llr,
                              uint8_t *d_syndrome, void *stream);

/* log((1. - q) / q) with the host C library, as src/qkd_ldpc_algorithm.cpp:1043. */
double qldpc_log_p(double qber);

/* keys_match = arrays_equal(alice, bob_solution) per frame
 * (src/qkd_ldpc_algorithm.cpp:1087; src/array_and_matrix_operations.cpp:105-118). */
int qldpc_keys_match_device(int32_t batch, int32_t n, const uint8_t *d_alice,
                            const uint8_t *d_bits, uint8_t *d_keys_match, void *stream);

/* The whole per-trial window of QKD_LDPC for `batch` trials on device: frame
 * construction + decode + key comparison.  d_synd_ws: caller-owned workspace
 * of batch*m bytes (Alice's syndromes).  d_llr_ws: batch*n doubles or NULL —
 * when given, the frames' LLRs are written there; NULL skips them where the
 * graph's decoder reads the frame builder's palette codes instead (the
 * register kernels), and uses an internal workspace otherwise. */
int qldpc_qkd_ldpc_batch_device(qldpc_graph *g, int32_t device, const qldpc_params *p,
                                int32_t batch, const uint8_t *d_alice, const uint8_t *d_bob,
                                const double *d_log_p, double *d_llr_ws, uint8_t *d_synd_ws,
                                uint8_t *d_bits_out, uint32_t *d_iters_out,
                                uint8_t *d_synd_ok_out, uint8_t *d_keys_match_out, void *stream);

/* --------------------------------------------------------------- introspection */

/* Launch geometry the decoder uses for this graph on `device`: lanes per frame
 * (threads per workgroup), edges per lane, resident workgroups, dynamic LDS
 * bytes and the kernel variant name (static string).  A host-only graph
 * (qldpc_graph_create_host) answers with workgroups == NULL. */
int qldpc_graph_plan(const qldpc_graph *g, int32_t device, int32_t algorithm, int32_t *lanes,
                     int32_t *edges_per_lane, int32_t *workgroups, int32_t *lds_bytes,
                     const char **variant);

/* Split-frame shape of the plan (n = 100k codes: a frame over several
 * workgroups of one XCD): parts per frame, lanes (threads) per part, and the
 * message slots per lane held in per-workgroup global scratch.  Frames of one
 * workgroup answer parts = 1 (part_lanes = the workgroup's lanes, scratch
 * slots of the hybrid shape included).  Any output pointer may be NULL. */
int qldpc_graph_split_plan(const qldpc_graph *g, int32_t *parts, int32_t *part_lanes, int32_t *scratch_slots);

/* The decoder's bank-aware label of every bit id (labels_out: n entries; the
 * identity when the plan keeps the reference's ids — split, hybrid and
 * first-generation shapes), and stats_out (nullable, 4 entries): summed LDS
 * bank excess of the slot layout before / after the relabelling search, and
 * the summed busiest-bank counts (LDS cycles of the slot groups) before / after.  Labels never change results: inputs and outputs
 * of every entry point use the reference's bit ids. */
int qldpc_graph_labels(const qldpc_graph *g, int32_t *labels_out, int64_t *stats_out);

/* Kernel timing: while enabled on g, every decode kernel launch is bracketed
 * by HIP events on the stream it runs on (nothing else: not the frame build,
 * the claim order or the key compare).  qldpc_last_decode_kernel_ms waits for
 * the last timed launch on (device, stream) and returns its duration in ms. */
int qldpc_set_kernel_timing(qldpc_graph *g, int32_t enabled);
int qldpc_last_decode_kernel_ms(qldpc_graph *g, int32_t device, void *stream, float *ms);

/* Diagnostic: the order in which the last decode on (device, stream) claimed
 * its frames (order.hip: ascending weight |H * z XOR s| of the channel
 * decision z) and each frame's weight, indexed by frame.  *count = the batch,
 * or 0 when that decode claimed frames in index order (QLDPC_ORDER=0, one
 * frame).  Waits for the stream.  No counterpart in the reference (its pool
 * decodes trials one at a time). */
int qldpc_last_claim_order(qldpc_graph *g, int32_t device, void *stream, int32_t *order_out, int32_t *weight_out,
                           int32_t cap, int32_t *count);

/* Diagnostic: evaluate the decoder's device math on `count` inputs on the
 * current device — fn 0 tanh, 1 atanh, 2 expm1, 3 log1p (exact_math.h, the
 * glibc-exact restatement), 4 tanh_lin_approx, 5 atanh_lin_approx
 * (src/qkd_ldpc_algorithm.cpp:146-172), 6 tanh and 7 atanh in the decoder
 * forms the SPA kernel calls, 8 tanh(x / 2.) in the table form of the SPA
 * check-node scan (tanh_half_clip_t; |x| >= 44 gives +-1), 9 clip(2. * atanh(x),
 * 100) in the SPA message pass's form (atanh2_clip). */
int qldpc_selftest_math_device(int32_t fn, int32_t count, const double *d_in, double *d_out, void *stream);

/* Thread-local description of the last failure on this thread. */
const char *qldpc_last_error(void);

/* Library version string. */
const char *qldpc_version(void);

/* Number of HIP devices visible to the process (the C++ drop-in's default
 * device list: every GPU of the node). */
int qldpc_device_count(int32_t *count);

/* ---- Trial generator ------------------------------------
 * qldpc_trial_seeds: the simulation loop's per-trial seeds — `count` draws of
 * uniform_int_distribution<size_t>(0, SIZE_MAX) over Xoshiro256PlusPlus(
 * simulation_seed) (src/simulation.cpp:713-719).  Host only.
 * qldpc_trials_device: for each trial f, run_trial's keys
 * (src/simulation.cpp:540-551): Alice = fill_random_bits, Bob = inject_errors
 * (src/array_and_matrix_operations.cpp:889-933) from a generator seeded with
 * d_seeds[f] + seed_add (the loop's `seeds[n] + curr_sim`, :743), with
 * libstdc++ 11's draw consumption.  d_alice/d_bob: batch*n bytes.  Returns
 * the accurate QBER floor(n*qber)/n; QLDPC_EINVAL (the reference's "too small
 * for QBER" error) when floor(n*qber) == 0. */
int qldpc_trial_seeds(uint64_t simulation_seed, int32_t count, uint64_t *seeds_out);
/* qldpc_xoshiro_jump: the Xoshiro256 state (s0..s3) of a generator seeded
 * like Xoshiro-cpp with `seed`, after `draws` draws, by the GF(2) jump matrix
 * the device trial generator starts its second wave from (draws = n: the state
 * after fill_random_bits).  Host only; the generator's self-check. */
int qldpc_xoshiro_jump(uint64_t seed, uint64_t draws, uint64_t *state_out);
int qldpc_trials_device(int32_t n, double qber, int32_t batch, const uint64_t *d_seeds, uint64_t seed_add,
                        uint8_t *d_alice, uint8_t *d_bob, double *accurate_qber_out, void *stream);

/* ---- Rate adaptation (a15) -----------------------------
 * qldpc_xoshiro_state: the 4-word state of Xoshiro256PlusPlus(seed).
 * qldpc_adapt_code_rate: adapt_code_rate (src/array_and_matrix_operations.cpp:
 * 1131-1223): numbers and ascending positions of punctured / shortened bits
 * for (qber, delta, efficiency), drawing from the generator whose state is
 * prng_state (advanced in place, so successive calls chain like the
 * reference's setup loop, src/simulation.cpp:394-455).  Untainted puncturing
 * takes the first positions of the .untp list.  Out-of-range combinations
 * (the reference's WARNING + skip) return QLDPC_OK with zero counts.
 * punctured_out / shortened_out need capacity n (NULL: counts only).
 * qldpc_rate_plan_create: the position classes of one (punctured, shortened)
 * pair, replicated on the graph's devices.
 * qldpc_trials_rate_adapt_device: qldpc_trials_device plus, per trial, the
 * 2 * n_punct further draws QKD_LDPC_RATE_ADAPT takes for punctured positions
 * (src/qkd_ldpc_algorithm.cpp:1148-1157) -> d_punct_alice/bob [batch*n_punct].
 * qldpc_build_frames_rate_adapt_device: the extended frame (:1141-1180):
 * Alice's extended key [batch*n], LLRs (+-log_p / 1e-4 / DBL_MAX) [batch*n]
 * and Alice's syndrome [batch*m].
 * qldpc_qkd_ldpc_rate_adapt_batch_device: QKD_LDPC_RATE_ADAPT's window on
 * device: frame build + decode + keys_match against the extended key (:1216);
 * d_llr_ws nullable as in qldpc_qkd_ldpc_batch_device. */
typedef struct qldpc_rate_plan qldpc_rate_plan;
int qldpc_xoshiro_state(uint64_t seed, uint64_t *state_out);
/* qldpc_select_punctured_untainted: select_punctured_bits_untainted
 * (src/array_and_matrix_operations.cpp:1002-1067, arXiv:1103.6149) — the
 * untainted puncturing list get_punctured_bits_untainted (:1076-1123) writes
 * to a missing .untp file, in selection order.  H as the flattened
 * check_nodes (row_ptr/col_idx) and bit_nodes (col_ptr/row_idx) lists; draws
 * from prng_state (advanced in place, as the reference's setup loop passes
 * its generator).  punctured_out needs capacity n (NULL: count only). */
int qldpc_select_punctured_untainted(int32_t n, int32_t m, const int32_t *row_ptr, const int32_t *col_idx,
                                     const int32_t *col_ptr, const int32_t *row_idx, uint64_t *prng_state,
                                     int32_t *punctured_out, int32_t *n_punctured);
int qldpc_adapt_code_rate(int32_t n, int32_t m, double qber, double delta, double efficiency,
                          int32_t untainted_enabled, const int32_t *untainted, int32_t n_untainted,
                          uint64_t *prng_state, int32_t *punctured_out, int32_t *n_punctured, int32_t *shortened_out,
                          int32_t *n_shortened, double *adapted_rate_out);
int qldpc_rate_plan_create(qldpc_graph *g, int32_t n_punct, const int32_t *punctured, int32_t n_short,
                           const int32_t *shortened, qldpc_rate_plan **out);
void qldpc_rate_plan_destroy(qldpc_rate_plan *plan);
int qldpc_trials_rate_adapt_device(int32_t n, double qber, int32_t batch, const uint64_t *d_seeds, uint64_t seed_add,
                                   int32_t n_punct, uint8_t *d_alice, uint8_t *d_bob, uint8_t *d_punct_alice,
                                   uint8_t *d_punct_bob, double *accurate_qber_out, void *stream);
int qldpc_build_frames_rate_adapt_device(qldpc_graph *g, const qldpc_rate_plan *plan, int32_t device, int32_t batch,
                                         const uint8_t *d_alice, const uint8_t *d_bob, const uint8_t *d_punct_alice,
                                         const uint8_t *d_punct_bob, const double *d_log_p, uint8_t *d_alice_ext,
                                         double *d_llr, uint8_t *d_syndrome, void *stream);
int qldpc_qkd_ldpc_rate_adapt_batch_device(qldpc_graph *g, const qldpc_rate_plan *plan, int32_t device,
                                           const qldpc_params *p, int32_t batch, const uint8_t *d_alice,
                                           const uint8_t *d_bob, const uint8_t *d_punct_alice,
                                           const uint8_t *d_punct_bob, const double *d_log_p, uint8_t *d_alice_ext,
                                           double *d_llr_ws, uint8_t *d_synd_ws, uint8_t *d_bits_out,
                                           uint32_t *d_iters_out, uint8_t *d_synd_ok_out, uint8_t *d_keys_match_out,
                                           void *stream);

/* ---- Simulation-driver helpers ----------------------
 * qldpc_sort_permutation: the order std::sort (libstdc++, not stable) leaves a
 * sequence in when comparing only `keys` — how the reference orders its
 * config maps by code_rate (src/config.cpp:43,289,355,389).
 * qldpc_bits_to_remove: privacy-maintenance bit positions
 * (get_bits_positions_to_remove / _rate_adapt,
 * src/array_and_matrix_operations.cpp:138-256), ascending; out needs capacity
 * n (NULL: count only).  The out-key length of the throughput columns is
 * n - count. */
int qldpc_sort_permutation(const double *keys, int32_t n, int32_t *perm_out);
int qldpc_bits_to_remove(int32_t n, int32_t m, const int32_t *col_ptr, const int32_t *row_idx, int32_t n_punct,
                         const int32_t *punctured, int32_t n_short, const int32_t *shortened, int32_t rate_adapt,
                         int32_t *out, int32_t *count);

/* ---- The simulation loop's batch seam --------------
 * qldpc_run_trials: run_trial for `count` trials of one combination
 * (src/simulation.cpp:540-576) — the body of QKD_LDPC_batch_simulation's
 * pool.detach_loop(0, TRIALS_NUMBER) (:721-746) — with host pointers only.
 * Trial t: a generator seeded with seeds[t] + seed_add (the loop's
 * `seeds[n] + curr_sim`), Alice = fill_random_bits, Bob = inject_errors
 * (src/array_and_matrix_operations.cpp:889-933), then QKD_LDPC (plan == NULL,
 * src/qkd_ldpc_algorithm.cpp:1031-1119) or QKD_LDPC_RATE_ADAPT with the plan's
 * punctured / shortened positions (:1121-1258, the punctured draws continuing
 * from the same generator).  Everything happens on device: only the seeds go
 * in and {iterations_num, syndromes_match, keys_match} per trial come back.
 * The trials are split in contiguous slices over the graph's devices, one
 * host thread each, no collectives; on each device chunks alternate over two
 * streams so the next chunk's trials are generated while one decodes.
 * runtime_us_out (nullable): trial_result::runtime — the measured duration of
 * the trial's chunk window (frame build + decode + key compare; trial
 * generation excluded, as :559-568 time only the QKD_LDPC call) shared out
 * over the chunk's trials in proportion to each trial's own decode span (its
 * frame's claim-to-result time on the GPU).  accurate_qber_out (nullable):
 * floor(n * qber) / n, every trial's trial_result::accurate_QBER.
 * Errors: QLDPC_EINVAL with run_trial's message when floor(n * qber) == 0. */
int qldpc_run_trials(qldpc_graph *g, const qldpc_rate_plan *plan, const qldpc_params *p, double qber,
                     int32_t count, const uint64_t *seeds, uint64_t seed_add, uint32_t *iters_out,
                     uint8_t *synd_ok_out, uint8_t *keys_match_out, double *runtime_us_out,
                     double *accurate_qber_out);
/* qldpc_run_trials in two halves, so the simulation loop can put combination
 * c + 1 on the devices before it collects combination c (the loop over
 * combinations, src/simulation.cpp:725-765): _submit checks the arguments
 * exactly as qldpc_run_trials, copies the seeds and enqueues the trials
 * (blocking only when both of a device's pipeline slots still hold chunks, which
 * it then collects for their own jobs), and returns a job; _wait completes the
 * job's outputs, frees it and returns the first error of any device slice.
 * Between the two the output arrays, the graph and the plan must stay alive;
 * the seeds need not.  Every submitted job must be waited for. */
typedef struct qldpc_trials_job qldpc_trials_job;
int qldpc_run_trials_submit(qldpc_graph *g, const qldpc_rate_plan *plan, const qldpc_params *p, double qber,
                            int32_t count, const uint64_t *seeds, uint64_t seed_add, uint32_t *iters_out,
                            uint8_t *synd_ok_out, uint8_t *keys_match_out, double *runtime_us_out,
                            double *accurate_qber_out, qldpc_trials_job **job_out);
int qldpc_run_trials_wait(qldpc_trials_job *job);
/* The device slice of the batch seam: trials [*lo, *hi) of `count` for shard
 * `shard` of `shards` (contiguous slices of ceil(count / shards); trailing
 * shards may be short or empty).  Host only. */
int qldpc_shard_range(int32_t count, int32_t shards, int32_t shard, int32_t *lo, int32_t *hi);

#ifdef __cplusplus
}
#endif
#endif
