/*
 * krr_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference
 * KRR v1.0.0 SimpleStrategy arithmetic, used as the parity checker for the
 * HIP path (tests/, __graft_entry__.smoke(), bench.py cpu_baseline leg).
 * The product path never links or calls this file.
 *
 * Parity status: PINNED.  tests/test_oracle_golden.py checks every function
 * here against golden vectors produced by importing the reference itself
 * (tests/golden/make_golden.py, run in the build container).
 *
 * Semantics restated (reference file:line under /root/reference):
 *  - segment = pods concatenated in dict order, each pod in timestamp order
 *    (robusta_krr/core/integrations/prometheus.py:150-155);
 *  - n = present samples; empty -> NaN (robusta_krr/strategies/simple.py:26-27, 33-34);
 *  - REF_INDEX: data_[int((n-1) * p / 100)] on the UNSORTED concatenation
 *    (simple.py:31-36); p = p_num/p_den, index computed exactly — or, for p whose
 *    28-digit Decimal product rounds, k = k_table[n] (oracle_percentile_ktab: the
 *    caller's table of the reference's own expression);
 *  - SORTED_LOWER: the same index into sorted(data_) — Python's sorted() is a
 *    stable sort under Decimal '<' (so -0 and +0 keep their input order);
 *  - LINEAR: numpy 2.2.6 np.percentile(method="linear"):
 *    numpy/lib/_function_base_impl.py _quantile / _get_indexes / _get_gamma / _lerp;
 *  - MAX: Python max() — the first element that no later element exceeds
 *    (simple.py:29); a NaN sample makes Decimal comparison raise, reported as
 *    KRR_FLAG_NAN.
 * NaN slots are absent samples when `gaps` is set (dense layout).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define FLAG_NAN 1u
#define FLAG_EMPTY 4u

enum { REF_INDEX = 0, SORTED_LOWER = 1, LINEAR = 2 };

static const double QNAN = __builtin_nan("");

/* floor((n-1) * p_num / (100 * p_den)) with 128-bit intermediates. */
int64_t oracle_exact_rank(int64_t n, int64_t p_num, int64_t p_den) {
    unsigned __int128 num = (unsigned __int128)(uint64_t)(n - 1) * (uint64_t)p_num;
    unsigned __int128 den = (unsigned __int128)100u * (uint64_t)p_den;
    return (int64_t)(num / den);
}

/* ---- stable merge sort under numeric '<' (Python sorted over Decimals) ---- */
static void merge_sort(double* a, double* tmp, int64_t n) {
    if (n < 2) return;
    int64_t h = n / 2;
    merge_sort(a, tmp, h);
    merge_sort(a + h, tmp, n - h);
    int64_t i = 0, j = h, k = 0;
    while (i < h && j < n) {
        /* take from the right only if strictly smaller: keeps stability */
        if (a[j] < a[i]) tmp[k++] = a[j++];
        else tmp[k++] = a[i++];
    }
    while (i < h) tmp[k++] = a[i++];
    while (j < n) tmp[k++] = a[j++];
    memcpy(a, tmp, (size_t)n * sizeof(double));
}

/* ---- quickselect under numeric '<' (numpy partition analogue) ---- */
static void swapd(double* a, double* b) {
    double t = *a;
    *a = *b;
    *b = t;
}
static double quickselect(double* a, int64_t n, int64_t k) {
    int64_t lo = 0, hi = n - 1;
    while (hi > lo) {
        int64_t mid = lo + (hi - lo) / 2;
        if (a[mid] < a[lo]) swapd(&a[mid], &a[lo]);
        if (a[hi] < a[lo]) swapd(&a[hi], &a[lo]);
        if (a[hi] < a[mid]) swapd(&a[hi], &a[mid]);
        double pv = a[mid];
        int64_t i = lo, j = hi;
        while (i <= j) {
            while (a[i] < pv) ++i;
            while (pv < a[j]) --j;
            if (i <= j) {
                swapd(&a[i], &a[j]);
                ++i;
                --j;
            }
        }
        if (k <= j) hi = j;
        else if (k >= i) lo = i;
        else return a[k];
    }
    return a[k];
}

/* numpy _lerp: a + (b-a)*t, or b - (b-a)*(1-t) where t >= 0.5; no FMA. */
static double np_lerp(double a, double b, double t) {
    volatile double d = b - a;
    if (t >= 0.5) {
        volatile double w = 1.0 - t;
        volatile double p = d * w;
        return b - p;
    }
    volatile double p = d * t;
    return a + p;
}

static int64_t gather_present(const double* v, int64_t beg, int64_t end, int gaps, double* out,
                              int64_t* nnan) {
    int64_t n = 0, nn = 0;
    for (int64_t i = beg; i < end; ++i) {
        double x = v[i];
        if (isnan(x)) {
            ++nn;
            if (gaps) continue;
        }
        out[n++] = x;
    }
    *nnan = nn;
    return n;
}

static int64_t rank_k(int64_t n, int64_t p_num, int64_t p_den, const int64_t* ktab) {
    return ktab ? ktab[n] : oracle_exact_rank(n, p_num, p_den);
}

static void one_percentile(const double* values, int64_t beg, int64_t end, int mode, int gaps,
                           int64_t p_num, int64_t p_den, const int64_t* ktab, double q, double* buf,
                           double* tmp, double* ov, int64_t* on, uint32_t* of) {
    int64_t nnan = 0;
    int64_t n = gather_present(values, beg, end, gaps, buf, &nnan);
    *on = n;
    *of = 0;
    if (n == 0) {
        *ov = QNAN;
        *of = FLAG_EMPTY;
        return;
    }
    if (mode == REF_INDEX) {
        *ov = buf[rank_k(n, p_num, p_den, ktab)];
        return;
    }
    if (nnan && !gaps) {
        *ov = QNAN;
        *of = FLAG_NAN;
        return;
    }
    if (mode == SORTED_LOWER) {
        merge_sort(buf, tmp, n);
        *ov = buf[rank_k(n, p_num, p_den, ktab)];
        return;
    }
    /* LINEAR, numpy: virtual index (n-1)*q, clip at n-1 with gamma vs index -1 */
    double vidx = (double)(n - 1) * q;
    int64_t prev, next;
    double gamma;
    if (vidx >= (double)(n - 1)) {
        prev = next = n - 1;
        gamma = vidx - (-1.0);
    } else {
        double fl = floor(vidx);
        prev = (int64_t)fl;
        next = prev + 1;
        gamma = vidx - fl;
    }
    double a = quickselect(buf, n, prev);
    double b = a;
    if (next != prev) {
        /* after quickselect, buf[prev+1..n) >= a: the next order statistic is their min */
        b = buf[next];
        for (int64_t i = next + 1; i < n; ++i)
            if (buf[i] < b) b = buf[i];
    }
    *ov = np_lerp(a, b, gamma);
}

/* k_table (may be NULL): k(n) = k_table[n], k_table_len > every segment's slots. */
int oracle_percentile_ktab(const double* values, const int64_t* offsets, int64_t S, int mode, int gaps,
                           int64_t p_num, int64_t p_den, const int64_t* k_table, int64_t k_table_len, double q,
                           double* out_v, int64_t* out_n, uint32_t* out_f, int nthreads) {
    if (mode < 0 || mode > 2 || p_den <= 0 || p_num <= 0) return -1;
    int64_t lmax = 0;
    for (int64_t s = 0; s < S; ++s) {
        int64_t L = offsets[s + 1] - offsets[s];
        if (L > lmax) lmax = L;
    }
    if (k_table && lmax >= k_table_len) return -3;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    int err = 0;
#pragma omp parallel
    {
        double* buf = (double*)malloc((size_t)(lmax > 0 ? lmax : 1) * sizeof(double));
        double* tmp = (double*)malloc((size_t)(lmax > 0 ? lmax : 1) * sizeof(double));
        if (!buf || !tmp) {
#pragma omp atomic write
            err = 1;
        } else {
#pragma omp for schedule(dynamic, 8)
            for (int64_t s = 0; s < S; ++s)
                one_percentile(values, offsets[s], offsets[s + 1], mode, gaps, p_num, p_den, k_table, q, buf,
                               tmp, &out_v[s], &out_n[s], &out_f[s]);
        }
        free(buf);
        free(tmp);
    }
    return err ? -2 : 0;
}

int oracle_percentile(const double* values, const int64_t* offsets, int64_t S, int mode, int gaps,
                      int64_t p_num, int64_t p_den, double q, double* out_v, int64_t* out_n,
                      uint32_t* out_f, int nthreads) {
    return oracle_percentile_ktab(values, offsets, S, mode, gaps, p_num, p_den, NULL, 0, q, out_v, out_n, out_f,
                                  nthreads);
}

int oracle_max(const double* values, const int64_t* offsets, int64_t S, int gaps, double* out_v,
               int64_t* out_n, uint32_t* out_f, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 8)
    for (int64_t s = 0; s < S; ++s) {
        int64_t n = 0, nn = 0;
        int have = 0;
        double cur = QNAN;
        for (int64_t i = offsets[s]; i < offsets[s + 1]; ++i) {
            double x = values[i];
            if (isnan(x)) {
                ++nn;
                if (gaps) continue;
                ++n;
                continue;
            }
            ++n;
            if (!have || x > cur) {
                cur = x;
                have = 1;
            }
        }
        out_n[s] = n;
        if (n == 0) {
            out_v[s] = QNAN;
            out_f[s] = FLAG_EMPTY;
        } else if (nn && !gaps) {
            out_v[s] = QNAN;
            out_f[s] = FLAG_NAN;
        } else {
            out_v[s] = cur;
            out_f[s] = 0;
        }
    }
    return 0;
}
