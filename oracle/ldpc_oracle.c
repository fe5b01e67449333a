/* ldpc_oracle.c — CPU ORACLE (test infrastructure only; see ldpc_oracle.h).
 *
 * Restates the reference decode loop of ColdCloudd/QKD_LDPC_V
 * src/qkd_ldpc_algorithm.cpp.  Data layout follows the reference's two message
 * matrices: B (bit_to_check_msg, indexed like check_nodes: row-major) and C
 * (check_to_bit_msg, indexed like bit_nodes: column-major), paired through the
 * reference's occurrence counters.  Math comes from the C library (tanh, atanh,
 * log, fabs), exactly as the reference's <cmath> calls.  Build with
 * -ffp-contract=off (oracle/Makefile).
 */
#include "ldpc_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

struct qlo_graph {
    int32_t n, m, E;
    int32_t *rowptr, *colidx; /* check_nodes */
    int32_t *colptr, *rowidx; /* bit_nodes */
    int32_t *cslot;           /* CN write slot in C for row-major edge e (check_pos_idx) */
    int32_t *rslot;           /* VN write slot in B for column-major edge f (bit_pos_idx) */
};

static int32_t *dup_i32(const int32_t *p, size_t k) {
    int32_t *q = (int32_t *)malloc((k ? k : 1) * sizeof(int32_t));
    if (q && k) memcpy(q, p, k * sizeof(int32_t));
    return q;
}

qlo_graph *qlo_graph_new(int32_t n, int32_t m, const int32_t *rowptr, const int32_t *colidx,
                         const int32_t *colptr, const int32_t *rowidx) {
    if (n <= 0 || m < 0 || rowptr[m] != colptr[n]) return NULL;
    const int32_t E = rowptr[m];
    qlo_graph *g = (qlo_graph *)calloc(1, sizeof(qlo_graph));
    g->n = n; g->m = m; g->E = E;
    g->rowptr = dup_i32(rowptr, (size_t)m + 1);
    g->colidx = dup_i32(colidx, (size_t)E);
    g->colptr = dup_i32(colptr, (size_t)n + 1);
    g->rowidx = dup_i32(rowidx, (size_t)E);
    g->cslot = (int32_t *)malloc(((size_t)E + 1) * sizeof(int32_t));
    g->rslot = (int32_t *)malloc(((size_t)E + 1) * sizeof(int32_t));
    int32_t *cnt_c = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    int32_t *cnt_r = (int32_t *)calloc((size_t)(m ? m : 1), sizeof(int32_t));
    int ok = 1;
    /* check_pos_idx: the k-th time bit i appears in the row-major CN traversal
     * it writes check_to_bit_msg[i][k] (src/qkd_ldpc_algorithm.cpp:67-69). */
    for (int32_t j = 0; j < m && ok; ++j)
        for (int32_t e = rowptr[j]; e < rowptr[j + 1]; ++e) {
            const int32_t i = colidx[e];
            if (i < 0 || i >= n || cnt_c[i] >= colptr[i + 1] - colptr[i]) { ok = 0; break; }
            g->cslot[e] = colptr[i] + cnt_c[i]++;
        }
    /* bit_pos_idx: the k-th time check j appears in the column-major VN traversal
     * it writes bit_to_check_msg[j][k] (src/qkd_ldpc_algorithm.cpp:116-118). */
    for (int32_t i = 0; i < n && ok; ++i)
        for (int32_t f = colptr[i]; f < colptr[i + 1]; ++f) {
            const int32_t j = rowidx[f];
            if (j < 0 || j >= m || cnt_r[j] >= rowptr[j + 1] - rowptr[j]) { ok = 0; break; }
            g->rslot[f] = rowptr[j] + cnt_r[j]++;
        }
    free(cnt_c);
    free(cnt_r);
    if (!ok) { qlo_graph_free(g); return NULL; }
    return g;
}

void qlo_graph_free(qlo_graph *g) {
    if (!g) return;
    free(g->rowptr); free(g->colidx); free(g->colptr); free(g->rowidx);
    free(g->cslot); free(g->rslot); free(g);
}

void qlo_syndrome(const qlo_graph *g, const uint8_t *bits, uint8_t *synd) {
    for (int32_t j = 0; j < g->m; ++j) {
        int s = 0;
        for (int32_t e = g->rowptr[j]; e < g->rowptr[j + 1]; ++e) s ^= bits[g->colidx[e]];
        synd[j] = (uint8_t)s;
    }
}

/* threshold_matrix, src/array_and_matrix_operations.cpp:953-972 (NaN passes). */
static void clip_all(double *v, int32_t E, double thr) {
    for (int32_t e = 0; e < E; ++e) {
        if (v[e] > thr) v[e] = thr;
        else if (v[e] < -thr) v[e] = -thr;
    }
}

/* Timing split only (tools/oracle_speed.py builds a copy with it defined): the
 * SPA's two C-library calls per edge replaced by sign-preserving stand-ins of
 * no cost, so the rest of the loop can be timed alone.  Never the oracle. */
#ifdef QLO_TIMING_NO_MATH
#define QLO_TANH(x) ((x) > 0. ? 0.6 : -0.6)
#define QLO_ATANH(x) ((x) * 3.)
#else
#define QLO_TANH(x) tanh(x)
#define QLO_ATANH(x) atanh(x)
#endif

/* tanh_lin_approx / atanh_lin_approx, src/qkd_ldpc_algorithm.cpp:146-172. */
static double tanh_lin(double x) {
    const double a = fabs(x);
    double r;
    if (a < 0.5) r = 0.9242 * a;
    else if (a < 0.9) r = 0.6355 * a + 0.1444;
    else if (a < 1.2) r = 0.3912 * a + 0.3642;
    else if (a < 1.75) r = 0.1958 * a + 0.5986;
    else if (a < 2.5) r = 0.0603 * a + 0.8358;
    else if (a < 3.5) r = 0.0115 * a + 0.9577;
    else if (a < 8) r = 0.0004 * a + 0.9967;
    else r = 1;
    return (x < 0.) ? -r : r;
}
static double atanh_lin(double x) {
    const double a = fabs(x);
    double r;
    if (a < 0.7) r = 1.196 * a - 0.0323;
    else if (a < 0.9) r = 2.9187 * a - 1.214;
    else if (a < 0.999) r = 10.8717 * a - 8.3717;
    else r = 2510.9 * a - 2505.9;
    return (x < 0.) ? -r : r;
}

static int32_t decode_impl(const qlo_graph *g, const qlo_params *p, const double *llr,
                           const uint8_t *synd, uint8_t *out, double *post, int32_t *synd_ok,
                           double *trace) {
    const int32_t n = g->n, m = g->m, E = g->E;
    const int alg = p->alg;
    const int adaptive = (alg == QLO_ANMSA || alg == QLO_AOMSA);
    double *B = (double *)malloc(((size_t)E + 1) * sizeof(double));
    double *C = (double *)calloc((size_t)E + 1, sizeof(double));
    double *total = (double *)calloc((size_t)n, sizeof(double));
    uint8_t *dsyn = (uint8_t *)calloc((size_t)(m ? m : 1), 1);
    int32_t result_it = p->max_iterations, matched = 0;

    /* bit_to_check_msg[j][k] = llr[check_nodes[j][k]] (unclipped), :21-29. */
    for (int32_t e = 0; e < E; ++e) B[e] = llr[g->colidx[e]];
    /* ANMSA/AOMSA start from the channel decision, :683-691. */
    if (adaptive)
        for (int32_t i = 0; i < n; ++i) out[i] = (llr[i] <= 0) ? 1 : 0;

    for (int32_t it = 0; it != p->max_iterations; ++it) {
        int all_eq = 1;
        /* ---- check-node update over all rows, in row order ---- */
        for (int32_t j = 0; j < m; ++j) {
            const int32_t e0 = g->rowptr[j], e1 = g->rowptr[j + 1];
            if (alg == QLO_SPA || alg == QLO_SPA_LIN) {
                double row_prod = synd[j] ? -1. : 1.;            /* :57 */
                for (int32_t e = e0; e < e1; ++e) {
                    B[e] = (alg == QLO_SPA) ? QLO_TANH(B[e] / 2.) : tanh_lin(B[e] / 2.);
                    row_prod *= B[e];
                }
                for (int32_t e = e0; e < e1; ++e) {
                    const double prod = row_prod / B[e];          /* :66 */
                    C[g->cslot[e]] = 2. * ((alg == QLO_SPA) ? QLO_ATANH(prod) : atanh_lin(prod));
                }
            } else {
                double sign_prod = synd[j] ? -1. : 1.;           /* :376 */
                int negative_count = 0;
                double min1 = DBL_MAX, min2 = DBL_MAX;
                for (int32_t e = e0; e < e1; ++e) {               /* :381-397 */
                    if (B[e] < 0) ++negative_count;
                    const double a = fabs(B[e]);
                    if (a < min1) { min2 = min1; min1 = a; }
                    else if (a < min2) { min2 = a; }
                }
                sign_prod *= (negative_count % 2 == 0) ? 1. : -1.;
                double factor = p->primary;
                if (adaptive) {                                   /* :745-757 */
                    int d = 0;
                    for (int32_t e = e0; e < e1; ++e) d ^= out[g->colidx[e]];
                    dsyn[j] = (uint8_t)d;
                    if (d != synd[j]) { factor = p->secondary; all_eq = 0; }
                }
                for (int32_t e = e0; e < e1; ++e) {
                    const double prod = sign_prod * ((B[e] > 0) ? 1. : -1.);   /* :402 */
                    const double sel = (fabs(B[e]) == min1) ? min2 : min1;
                    if (alg == QLO_NMSA || alg == QLO_ANMSA) {
                        C[g->cslot[e]] = factor * prod * sel;                 /* :405-406 */
                    } else {
                        const double diff = sel - factor;                      /* :573-574 */
                        C[g->cslot[e]] = prod * ((diff < 0.) ? 0. : diff);
                    }
                }
            }
        }
        /* ANMSA/AOMSA exit right after the CN pass, :770-776 / :960-966. */
        if (adaptive && all_eq) { result_it = it + 1; matched = 1; break; }

        if (p->thr_enabled) clip_all(C, E, p->thr);                       /* :73-74 */

        /* ---- totals + hard decision, std::accumulate order, :76-84 ---- */
        for (int32_t i = 0; i < n; ++i) {
            double acc = llr[i];
            for (int32_t f = g->colptr[i]; f < g->colptr[i + 1]; ++f) acc = acc + C[f];
            total[i] = acc;
            out[i] = (acc <= 0) ? 1 : 0;
        }
        if (trace) memcpy(trace + (size_t)it * n, total, (size_t)n * sizeof(double));

        if (!adaptive) {                                                  /* :86,101-107 */
            qlo_syndrome(g, out, dsyn);
            int eq = 1;
            for (int32_t j = 0; j < m; ++j)
                if (dsyn[j] != synd[j]) { eq = 0; break; }
            if (eq) { result_it = it + 1; matched = 1; break; }
        }
        /* ---- extrinsic bit-to-check messages, :109-120 ---- */
        for (int32_t i = 0; i < n; ++i) {
            const double col_sum = total[i];
            for (int32_t f = g->colptr[i]; f < g->colptr[i + 1]; ++f) B[g->rslot[f]] = col_sum - C[f];
        }
        if (p->thr_enabled) clip_all(B, E, p->thr);                       /* :122-123 */
    }
    if (post) memcpy(post, total, (size_t)n * sizeof(double));
    if (synd_ok) *synd_ok = matched;
    free(B); free(C); free(total); free(dsyn);
    return result_it;
}

int32_t qlo_decode(const qlo_graph *g, const qlo_params *p, const double *llr, const uint8_t *synd,
                   uint8_t *out, double *post, int32_t *synd_ok) {
    return decode_impl(g, p, llr, synd, out, post, synd_ok, NULL);
}

int32_t qlo_decode_trace(const qlo_graph *g, const qlo_params *p, const double *llr,
                         const uint8_t *synd, uint8_t *out, double *post, int32_t *synd_ok,
                         double *trace_post) {
    return decode_impl(g, p, llr, synd, out, post, synd_ok, trace_post);
}

typedef struct {
    const qlo_graph *g; const qlo_params *p; int32_t batch; const double *llr; const uint8_t *synd;
    uint8_t *out; uint32_t *iters; uint8_t *ok; double *post;
    int32_t next; pthread_mutex_t mu;
} batch_job;

static void *batch_worker(void *arg) {
    batch_job *J = (batch_job *)arg;
    const size_t n = (size_t)J->g->n, m = (size_t)J->g->m;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        const int32_t f = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (f >= J->batch) break;
        int32_t ok = 0;
        const int32_t it = decode_impl(J->g, J->p, J->llr + f * n, J->synd + f * m, J->out + f * n,
                                       J->post ? J->post + f * n : NULL, &ok, NULL);
        if (J->iters) J->iters[f] = (uint32_t)it;
        if (J->ok) J->ok[f] = (uint8_t)ok;
    }
    return NULL;
}

void qlo_decode_batch(const qlo_graph *g, const qlo_params *p, int32_t batch, const double *llr,
                      const uint8_t *synd, uint8_t *out, uint32_t *iters, uint8_t *synd_ok,
                      double *post, int32_t threads) {
    batch_job J = {g, p, batch, llr, synd, out, iters, synd_ok, post, 0, PTHREAD_MUTEX_INITIALIZER};
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    for (int32_t t = 0; t < threads; ++t) pthread_create(&th[t], NULL, batch_worker, &J);
    for (int32_t t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(th);
}

void qlo_build_frame(const qlo_graph *g, const uint8_t *alice, const uint8_t *bob, double qber,
                     double *llr, uint8_t *synd) {
    const double log_p = log((1. - qber) / qber);                          /* :1043 */
    for (int32_t i = 0; i < g->n; ++i) llr[i] = bob[i] ? -log_p : log_p;   /* :1046-1049 */
    qlo_syndrome(g, alice, synd);                                          /* :1051-1052 */
}

int32_t qlo_qkd_ldpc(const qlo_graph *g, const qlo_params *p, const uint8_t *alice,
                     const uint8_t *bob, double qber, uint8_t *bob_solution,
                     int32_t *synd_ok, int32_t *keys_match) {
    double *llr = (double *)malloc((size_t)g->n * sizeof(double));
    uint8_t *s = (uint8_t *)malloc((size_t)(g->m ? g->m : 1));
    qlo_build_frame(g, alice, bob, qber, llr, s);
    const int32_t it = qlo_decode(g, p, llr, s, bob_solution, NULL, synd_ok);
    int eq = 1;                                                            /* arrays_equal, :1087 */
    for (int32_t i = 0; i < g->n; ++i)
        if (alice[i] != bob_solution[i]) { eq = 0; break; }
    if (keys_match) *keys_match = eq;
    free(llr); free(s);
    return it;
}
