/*
 * krr_amd.h — C ABI of the MI355X-native KRR SimpleStrategy hot path.
 *
 * The reference (KRR v1.0.0) computes, per Kubernetes object, a CPU "percentile"
 * and a memory max over Prometheus range-query series, one object at a time in
 * Python Decimal.  This ABI replaces that per-object work with fleet-wide
 * segmented kernels over one CSR float64 buffer:
 *
 *   segment s  = one (object, resource) series: the concatenation of the
 *                object's pods in K8sObjectData.pods order, each pod's samples
 *                in timestamp order (reference core/integrations/prometheus.py:150-155).
 *   values[]   = float64 samples of every segment, back to back.
 *   offsets[]  = S+1 int64 offsets; segment s is values[offsets[s] .. offsets[s+1]).
 *
 * A NaN slot is an ABSENT sample when `gaps_are_nan` is set (dense layout
 * with pods aligned on a time grid); otherwise NaN is a real sample value
 * and follows the reference's NaN behaviour (see KRR_FLAG_NAN).
 *
 * Entry points and the reference interface each replaces:
 *
 *   krr_segmented_percentile  <- SimpleStrategySettings.calculate_cpu_proposal
 *                                robusta_krr/strategies/simple.py:31-36
 *   krr_segmented_max         <- SimpleStrategySettings.calculate_memory_proposal
 *                                robusta_krr/strategies/simple.py:24-29 (the max;
 *                                the x(1+b/100) buffer is exact-decimal host work)
 *   krr_simple_run            <- SimpleStrategy.run robusta_krr/strategies/simple.py:42-49,
 *                                batched over every object (the loop the reference
 *                                runs in Runner._gather_objects_recommendations,
 *                                robusta_krr/core/runner.py:88-120)
 *   krr_simple_run_host       <- same, for callers holding host buffers (PCIe-inclusive)
 *   krr_json_parse / _compact <- PrometheusLoader.gather_data's per-pod value parse,
 *                                robusta_krr/core/integrations/prometheus.py:147-155,
 *                                on response bodies in HBM (device packer)
 *   krr_json_find_series / _parse_segments / _gather
 *                             <- the same for grouped `sum by (pod)` bodies (the fleet
 *                                batching of prometheus.py:118-143's per-pod queries)
 *
 * Ownership: the caller owns every buffer; no allocation crosses the ABI.
 * Device pointers are HIP device pointers on the ctx's device; `stream` is a
 * hipStream_t (NULL = default stream).  Calls are asynchronous on `stream`
 * unless stated.  Functions return KRR_OK (0) or a negative krr_status and
 * never throw; krr_last_error(ctx) returns the message of the last failure.
 * A ctx is not shared between threads (one ctx per thread/device); there is
 * no global mutable state, so distinct ctxs are reentrant.
 */
#ifndef KRR_AMD_H
#define KRR_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KRR_ABI_VERSION 3  /* 3: krr_percentile_params gained k_table / k_table_len;
                              2: krr_kll_params gained `tail`; krr_kll_merge; krr_kll_query takes series_base */

typedef enum {
    KRR_OK = 0,
    KRR_E_INVALID = -1,     /* bad argument (null pointer, bad mode, p out of (0,100]) */
    KRR_E_HIP = -2,         /* HIP runtime error (message in krr_last_error) */
    KRR_E_CAPACITY = -3,    /* a segment needs more selection scratch than was provisioned */
    KRR_E_UNSUPPORTED = -4, /* option combination not implemented */
    KRR_E_TIMEOUT = -5      /* a bounded wait ran out (krr_comm_init_timeout) */
} krr_status;

/* Percentile rule for the CPU recommendation.  All rules share n = number of
 * present samples and, for the exact rules, the index k(n).  The reference
 * evaluates k = int((n-1) * p / 100) (simple.py:36) in Decimal (prec 28, CLI path)
 * or in int arithmetic (the default int 99).  That equals the exact floor
 * floor((n-1) * p_num / p_den / 100), which the kernels compute in 128-bit
 * integers, whenever (n-1) * p has at most 28 significant digits; past that the
 * product is ROUNDED before the floor (p = 99.99999999999999999999999999 gives
 * k(3) = 2, not 1).  For such p the caller evaluates the reference's expression
 * per n and passes it as krr_percentile_params.k_table. */
typedef enum {
    KRR_PCT_REF_INDEX = 0,    /* X[k] of the UNSORTED pod-ordered concatenation (the
                                 reference's actual rule, simple.py:36) */
    KRR_PCT_SORTED_LOWER = 1, /* sorted(X)[k]  (stable sort, README.md:103 intent) */
    KRR_PCT_LINEAR = 2        /* np.percentile(X, p, method="linear") bit-exact:
                                 vidx=(n-1)*q in f64, numpy _lerp without FMA */
} krr_percentile_mode;

/* Per-segment flags written to out_flags. */
#define KRR_FLAG_NAN 1u       /* a NaN sample was present (gaps_are_nan == 0): the
                                 reference raises decimal.InvalidOperation for max()
                                 and sorted(); numpy returns NaN */
#define KRR_FLAG_CAPACITY 2u  /* internal selection bound violated (never expected) */
/* bits 8..15 of a KRR_FLAG_CAPACITY result carry an internal reason code (diagnostic) */
#define KRR_FLAG_EMPTY 4u     /* n == 0: value is NaN (reference: Decimal('NaN'),
                                 simple.py:26-27 and 33-34) */
#define KRR_FLAG_SKETCH_RANGE 8u /* sketch mode: a needed rank fell in a lumped bin
                                    (negative, below 2^min_exponent, or above the
                                    binned octaves): the value is a coarse estimate */

typedef struct {
    const double* values;    /* device pointer, n_values float64 */
    const int64_t* offsets;  /* device pointer, n_segments+1 int64, non-decreasing */
    int64_t n_segments;
    int64_t n_values;
    int64_t max_segment_len; /* upper bound on offsets[s+1]-offsets[s]; 0 = compute it (syncs) */
    int32_t gaps_are_nan;    /* 1: NaN slot = absent sample */
    int32_t reserved;
} krr_series;

typedef struct {
    int32_t mode;            /* krr_percentile_mode */
    int32_t reserved;
    int64_t p_num;           /* percentile p = p_num / p_den exactly, 0 < p <= 100 */
    int64_t p_den;           /* positive; p_den <= 1e15 (with k_table: a rational within 1e-15
                                of p, used only to size selection buffers) */
    double q;                /* float64(p) / 100.0 as numpy computes it (LINEAR only) */
    /* Optional index table (REF_INDEX / SORTED_LOWER; LINEAR ignores it): k(n) =
     * k_table[n] for 1 <= n < k_table_len, device-accessible (HBM or page-locked host
     * memory).  NULL: k(n) = the exact floor above.  Entries outside [0, n-1] are clamped
     * into it.  k_table_len must exceed the longest segment's slots (checked, KRR_E_INVALID)
     * or, for sketch / KLL / window queries, every merged present count (a series past the
     * table is flagged KRR_FLAG_CAPACITY). */
    const int64_t* k_table;
    int64_t k_table_len;
} krr_percentile_params;

typedef struct krr_ctx krr_ctx;

int krr_abi_version(void);

/* Create a context bound to HIP device `device` (a process may hold several). */
int krr_create(int device, krr_ctx** out_ctx);
int krr_destroy(krr_ctx* ctx);
const char* krr_last_error(const krr_ctx* ctx);

/* CPU proposal per segment.  out_value[s] = the selected f64 sample (bit-exact),
 * out_count[s] = n (present samples), out_flags[s] = KRR_FLAG_*.  All outputs are
 * device pointers with n_segments entries. */
int krr_segmented_percentile(krr_ctx* ctx, const krr_series* series,
                             const krr_percentile_params* params, double* out_value,
                             int64_t* out_count, uint32_t* out_flags, void* stream);

/* Memory proposal per segment: out_value[s] = max(X) with Python max() tie rule
 * (first maximal element, which only matters for -0.0 vs +0.0), out_count[s] = n. */
int krr_segmented_max(krr_ctx* ctx, const krr_series* series, double* out_value,
                      int64_t* out_count, uint32_t* out_flags, void* stream);

/* SimpleStrategy.run over every object: cpu and mem each hold one segment per
 * object (same n_segments).  Outputs are device pointers of n_segments entries. */
int krr_simple_run(krr_ctx* ctx, const krr_series* cpu, const krr_series* mem,
                   const krr_percentile_params* params, double* cpu_value, int64_t* cpu_count,
                   uint32_t* cpu_flags, double* mem_value, int64_t* mem_count,
                   uint32_t* mem_flags, void* stream);

/* krr_simple_run that also writes each object's 32-byte result record
 * (krr_pack_records layout: cpu bits, mem bits, cpu count | cpu flags << 48,
 * mem count | mem flags << 48) from the same launch — no separate pack pass.
 * records: device-accessible int64[4 * n_objects] — HBM, or page-locked host memory
 * (hipHostMalloc / a pinned torch tensor: mapped into the device's address space, so
 * the launch writes the records to the host itself and no D2H copy follows) — or NULL
 * (= krr_simple_run).  Host records are complete once the stream has synchronised. */
int krr_simple_run_records(krr_ctx* ctx, const krr_series* cpu, const krr_series* mem,
                           const krr_percentile_params* params, double* cpu_value, int64_t* cpu_count,
                           uint32_t* cpu_flags, double* mem_value, int64_t* mem_count, uint32_t* mem_flags,
                           int64_t* records, void* stream);

/* krr_simple_run_records whose launch also copies forward_bytes (a multiple of 16;
 * 16-byte aligned pointers) from forward_src to forward_dst: device memory, or
 * page-locked host memory mapped into the device's address space.  The copy runs as
 * the first work items of the same launch, beside the HBM stream, instead of as a
 * separate copy after it.  Multi-GPU step on the root: forward the previous step's
 * gathered records (N x 32 B per object) to the host while this step's pass runs —
 * no second stream, no cross-stream wait.  forward_bytes = 0: krr_simple_run_records.
 * (Compact REF_INDEX, which is not fused, or zero objects: a stream-ordered copy.) */
int krr_simple_run_forward(krr_ctx* ctx, const krr_series* cpu, const krr_series* mem,
                           const krr_percentile_params* params, double* cpu_value, int64_t* cpu_count,
                           uint32_t* cpu_flags, double* mem_value, int64_t* mem_count, uint32_t* mem_flags,
                           int64_t* records, const void* forward_src, void* forward_dst, int64_t forward_bytes,
                           void* stream);

/* Same as krr_simple_run, but every pointer (inputs and outputs) is a HOST
 * pointer; copies in, runs, copies out and synchronises.  Includes PCIe. */
int krr_simple_run_host(krr_ctx* ctx, const double* cpu_values, const int64_t* cpu_offsets,
                        const double* mem_values, const int64_t* mem_offsets,
                        int64_t n_objects, int32_t gaps_are_nan,
                        const krr_percentile_params* params, double* cpu_value,
                        int64_t* cpu_count, uint32_t* cpu_flags, double* mem_value,
                        int64_t* mem_count, uint32_t* mem_flags);

/* Multi-GPU result records: int64[4] per object (32 B) = cpu value bits, mem value
 * bits, cpu count | cpu flags << 48, mem count | mem flags << 48.  Device pointers;
 * records has 4 * n_objects entries.  (What a rank sends to rank 0 over RCCL.) */
int krr_pack_records(krr_ctx* ctx, int64_t n_objects, const double* cpu_value,
                     const int64_t* cpu_count, const uint32_t* cpu_flags, const double* mem_value,
                     const int64_t* mem_count, const uint32_t* mem_flags, int64_t* records,
                     void* stream);

/* ---- Multi-GPU result collection: RCCL over xGMI, one process per GPU ----
 * Replaces the reference's fleet fan-out (asyncio.gather over objects,
 * robusta_krr/core/runner.py:109-120) once the fleet is sharded over ranks: every
 * rank runs krr_simple_run_records on its contiguous object range, then the
 * records meet on the root.  RCCL is resolved at run time: the librccl.so.1
 * already loaded in the process (e.g. PyTorch's, so a communicator taken from a
 * torch.distributed "nccl" process group works) or else ROCm's.  `comm` is an
 * ncclComm_t.  Returns KRR_E_UNSUPPORTED when no RCCL can be loaded. */

/* unique_id: 128 bytes (ncclUniqueId), created on one rank and shared out of band. */
int krr_comm_unique_id(krr_ctx* ctx, void* unique_id);
/* ncclCommInitRank on the ctx's device. */
int krr_comm_init(krr_ctx* ctx, int nranks, const void* unique_id, int rank, void** out_comm);
/* The same, bounded: a nonblocking communicator (ncclCommInitRankConfig, blocking = 0) whose
 * state is polled for up to timeout_s seconds; when a peer never arrives the communicator is
 * aborted (ncclCommAbort) and KRR_E_TIMEOUT is returned instead of hanging.  Calls on the
 * communicator then wait for its state themselves (krr_gather_results does).  timeout_s <= 0:
 * krr_comm_init. */
int krr_comm_init_timeout(krr_ctx* ctx, int nranks, const void* unique_id, int rank, double timeout_s,
                          void** out_comm);
int krr_comm_destroy(krr_ctx* ctx, void* comm);

/* The communicator's rank count and this process's rank in it (ncclCommCount /
 * ncclCommUserRank): what a multi-GPU run reports to show RCCL carried every rank. */
int krr_comm_info(krr_ctx* ctx, void* comm, int* nranks, int* rank);

/* Gather every rank's n_local records (device int64[4 * n_local]) to `root`,
 * concatenated in rank order into `out` (device, root only; ignored elsewhere).
 * counts: HOST int64[nranks] with every rank's n_local, read on the root only; NULL
 * means every rank sends the root's n_local.  One grouped send/recv round (ragged
 * shards need no padding); asynchronous on `stream`. */
int krr_gather_results(krr_ctx* ctx, void* comm, int root, const int64_t* records, int64_t n_local,
                       const int64_t* counts, int64_t* out, void* stream);

/* ---- Launch plan (host only: no device, no ctx) ----
 * What krr_segmented_percentile (and, in fused_hselect, krr_simple_run) chooses for
 * SORTED_LOWER / LINEAR when the longest segment has max_segment_len slots.  The
 * other fields describe the krr_segmented_percentile launch. */
typedef struct {
    int32_t hselect;      /* 1: window select (wselect; hselect for its misses); 0: single-pass LDS candidate buffer */
    int32_t bottom;       /* 1: the smallest keys are kept (low percentiles) */
    int64_t tkeep;        /* keys a segment of max length must keep */
    int64_t cap_keys;     /* single-pass candidate capacity (0 with hselect) */
    int64_t lds_bytes;    /* dynamic LDS per workgroup (compact layout; a gapped one keeps the short-segment window) */
    int32_t probe;        /* 1: a max-length segment starts at a probe-estimated threshold */
    int32_t fused_hselect; /* the same choice for krr_simple_run's fused launch */
} krr_select_plan_info;

int krr_select_plan(int64_t max_segment_len, const krr_percentile_params* params, krr_select_plan_info* out);

/* Counters of the ctx since krr_create (synchronises the device): segments whose
 * one-pass window select (wselect) missed and were finished by the two-pass
 * histogram select.  Diagnostic: results are exact either way. */
int krr_get_stats(krr_ctx* ctx, int64_t* wselect_fallbacks);

/* ---- Sketch mode (config 5: time-sharded series too long for one window) ----
 * A build-only extension: the reference cannot query 30d@15s.
 * Per segment a log-linear histogram with data-independent bins: 2^mantissa_bits
 * bins per octave over [2^min_exponent, 2^(min_exponent+octaves)), plus four
 * lumped bins (negative, +-0, below range, above range).  Sketches of the same
 * series' time slices on different ranks merge exactly by adding counts (and
 * min/max by min/max); the query interpolates inside the bin holding the rank.
 * Its rank error is reported by the caller (bench.py config 5), not assumed. */
typedef struct {
    int32_t mantissa_bits;   /* m in [0, 10]: relative bin width <= 2^-m */
    int32_t min_exponent;    /* lowest binned octave [2^e, 2^(e+1)); e >= -1022 */
    int32_t octaves;         /* binned octaves; min_exponent + octaves <= 1024 */
    int32_t reserved;
} krr_sketch_params;

/* uint32 words per segment sketch: (octaves << mantissa_bits) + 4, or < 0 if invalid. */
int64_t krr_sketch_width(const krr_sketch_params* sp);

/* counts[S * width] (uint32), vmin/vmax[S] (NaN when empty), flags[S] (KRR_FLAG_NAN
 * when a NaN sample is present and gaps_are_nan == 0).  Device pointers. */
int krr_sketch_build(krr_ctx* ctx, const krr_series* series, const krr_sketch_params* sp,
                     uint32_t* counts, double* vmin, double* vmax, uint32_t* flags, void* stream);

/* Percentile from (merged) sketches: SORTED_LOWER or LINEAR over n = sum(counts).
 * out_flags: KRR_FLAG_EMPTY, KRR_FLAG_SKETCH_RANGE.  REF_INDEX -> KRR_E_UNSUPPORTED
 * (use krr_select_present on the time-sharded slices instead: it is exact). */
int krr_sketch_query(krr_ctx* ctx, int64_t n_segments, const uint32_t* counts, const double* vmin,
                     const double* vmax, const krr_sketch_params* sp, const krr_percentile_params* params,
                     double* out_value, int64_t* out_count, uint32_t* out_flags, void* stream);

/* ---- KLL sketch (row format 2): a RANK-error bound whatever the data, an exact top tail,
 * and a bounded fold ----
 * (north_star: "an optional mergeable t-digest/KLL sketch mode"; the log-linear sketch above
 * bounds the value error only.)  Specification: oracle/kll_ref.py; layout and schedule:
 * krr_amd/csrc/krr_kll.h.  One HBM pass per series slice builds one row of
 * krr_kll_row_words() uint64 words:
 *   - body: a compactor hierarchy with a DETERMINISTIC schedule — every compaction takes an
 *     even number of equal-weight keys (an odd largest key waits in its level's odd slot), so
 *     level sizes and sum(w^2) (row word 4) depend on the input's presence pattern only, and
 *     the total weight equals the present count exactly.  With probability >= 1 - delta every
 *     body answer's rank is within sqrt(2 ln(4/delta) sum(w^2)) of the asked rank
 *     (Azuma-Hoeffding; krr_amd.core.sketch.kll_rank_bound).  At most `budget` keys.
 *   - tail: the `tail` largest present keys, exactly: a rank r with n - r <= min(n, tail)
 *     (e.g. p99 of 172,800 samples with tail >= 1,729) is answered exactly.
 * Rows of one series (time slices, days, ...) FOLD into one row of the same size
 * (krr_kll_merge): counts add, the tails keep the `tail` largest of their union, the body
 * levels are unioned and compacted from level 0 up until `budget` keys remain. */
typedef struct {
    int32_t budget;   /* body keys per row: [256, 4096], a multiple of 64 */
    int32_t slice;    /* build: this slice's index (coin key); merge / query: the fold epoch */
    uint64_t seed;    /* coins: (seed, series, slice or epoch, event) hashed */
    int32_t tail;     /* exact tail keys per row: [0, 4096] */
    int32_t reserved; /* flags: KRR_KLL_ONE_PASS_TAIL (build); 0 otherwise */
} krr_kll_params;

/* krr_kll_params.reserved: keep the tail inside the build's one pass (a running buffer of
 * candidates above a rising threshold) instead of the default second pass over the slice
 * (candidates above a threshold read from the row's own body).  Rows are identical. */
#define KRR_KLL_ONE_PASS_TAIL 1
/* Testing: the tail pass's threshold without its rank-bound margin, so the body's estimate
 * often keeps fewer than `tail` keys and the pass streams the slice again (same rows). */
#define KRR_KLL_TAIL_NO_MARGIN 2
/* Build only the body: the tail words stay zero (word 6 = 0) until krr_kll_tail fills them
 * (callers that time the two passes apart, e.g. bench.py). */
#define KRR_KLL_BODY_ONLY 4

/* uint64 words per row (16 + budget + tail), or < 0 if invalid. */
int64_t krr_kll_row_words(const krr_kll_params* kp);

/* rows[S * row_words] (device): one row per segment of `series` (gaps_are_nan respected:
 * NaN gaps are absent; a NaN sample in the compact layout is counted in row word 1).
 * tail > 0: two launches on `stream` (k_kll_build, then k_kll_tail reading the slice again)
 * unless KRR_KLL_ONE_PASS_TAIL; the tail pass needs max((tail + 1,152) x 8,
 * (16 + budget) x 8 + budget) bytes of LDS.
 * seg_base: global index of segment 0 (coins depend on it).  KRR_E_UNSUPPORTED for
 * segments past ~130 M slots (run levels). */
int krr_kll_build(krr_ctx* ctx, const krr_series* series, const krr_kll_params* kp, int64_t seg_base,
                  uint64_t* rows, void* stream);

/* The tail pass alone, on rows krr_kll_build wrote with KRR_KLL_BODY_ONLY (same series, same
 * params): fills each row's tail words and word 6.  No-op when kp->tail == 0. */
int krr_kll_tail(krr_ctx* ctx, const krr_series* series, const krr_kll_params* kp, uint64_t* rows, void* stream);

/* The sparse two-pass form (round 5): the body build also records, per 16-slot line (128 B) of
 * the slice, an upper bound of its largest present key (32 bits of the order-preserving key,
 * rounded up); the tail pass then reads only the lines whose bound reaches its threshold
 * (candidates: the keys above the body's estimate of the tail's start) — about a fifth of the
 * slice at p99 of 30d@15s, instead of all of it.  Rows equal krr_kll_build's bit for bit.
 * lines: caller-owned device uint32 [n_segments * line_stride], line_stride >=
 * krr_kll_line_words(max_segment_len) (64 words per 1,024 slots, about 1/32 of the values'
 * bytes).  krr_kll_build_lines: the body-only build (tail > 0; leaves the tail words zero);
 * krr_kll_tail_lines: the tail pass that reads them; lines_read (optional device uint32
 * [n_segments]) gets the 128-B lines it read per segment (a whole-slice restream counts all). */
int64_t krr_kll_line_words(int64_t max_segment_len);
int krr_kll_build_lines(krr_ctx* ctx, const krr_series* series, const krr_kll_params* kp, int64_t seg_base,
                        uint64_t* rows, uint32_t* lines, int64_t line_stride, void* stream);
int krr_kll_tail_lines(krr_ctx* ctx, const krr_series* series, const krr_kll_params* kp, uint64_t* rows,
                       const uint32_t* lines, int64_t line_stride, uint32_t* lines_read, void* stream);

/* Fold each series' rows_per_series rows (rows[(s * W + w) * row_words], e.g. its W time
 * slices after an all-to-all, in time order) left to right into ONE row out_rows[s * row_words]
 * of the same format: coins keyed by (kp->seed, series_base + s, kp->slice as the epoch, w).
 * LDS per series: (3 row_words + 5 budget) x 8 bytes, whatever rows_per_series is (the fold
 * is left to right, one row at a time); KRR_E_CAPACITY when that exceeds the device's LDS
 * (160 KiB on gfx950).  With the query's extra budget bytes, rows that both fold and query
 * satisfy 24 (16 + budget + tail) + 41 budget <= 163,840: budget 512 with any tail, 1024 with
 * tail <= 4,037, 2048 with tail <= 1,264; budget 4096 builds but cannot fold. */
int krr_kll_merge(krr_ctx* ctx, int64_t n_series, int32_t rows_per_series, const uint64_t* rows,
                  const krr_kll_params* kp, int64_t series_base, uint64_t* out_rows, void* stream);

/* Percentile of every series from its rows (folded as krr_kll_merge first when W > 1):
 * SORTED_LOWER or LINEAR over n = present samples; rank 0 and n - 1: the exact min / max;
 * n - r <= tail length: the exact tail key; else the smallest body key whose weighted count
 * of keys <= it exceeds r.  out_flags: KRR_FLAG_EMPTY, KRR_FLAG_NAN (value NaN),
 * KRR_FLAG_CAPACITY (a row overflowed its levels or formats differ; never expected).
 * LDS as krr_kll_merge plus budget bytes (the same KRR_E_CAPACITY rule, independent of
 * rows_per_series).  REF_INDEX -> KRR_E_UNSUPPORTED. */
int krr_kll_query(krr_ctx* ctx, int64_t n_series, int32_t rows_per_series, const uint64_t* rows,
                  const krr_kll_params* kp, int64_t series_base, const krr_percentile_params* params,
                  double* out_value, int64_t* out_count, uint32_t* out_flags, void* stream);

/* ---- Exact refinement of merged sketches (config 5, exact percentiles) ----
 * The merged counts are exact, so they locate each needed rank's bin exactly:
 *   1. krr_sketch_locate on the owner's merged sketches -> krr_sketch_loc per series;
 *   2. every rank: krr_sketch_range_count (its local sketch) sizes, and
 *      krr_sketch_collect fills, the CSR of its samples inside [bin_lo, bin_hi];
 *   3. the owner concatenates the ranks' lists in time order (RCCL all-to-all) and
 *      krr_sketch_refine selects the ranks inside them: the exact SORTED_LOWER /
 *      LINEAR result (bit-identical to krr_segmented_percentile on the whole series). */
typedef struct {
    int64_t n;               /* present samples of the series (sum of merged counts) */
    int64_t r0, r1;          /* ascending ranks needed (0-based); r1 == r0 for SORTED_LOWER */
    int64_t before;          /* samples in bins below bin_lo */
    double gamma;            /* LINEAR weight (numpy method="linear") */
    uint32_t bin_lo, bin_hi; /* bins holding r0 and r1; bin_lo > bin_hi (empty) when n == 0 */
    uint32_t flags;          /* KRR_FLAG_EMPTY */
    int32_t mode;            /* KRR_PCT_SORTED_LOWER or KRR_PCT_LINEAR */
} krr_sketch_loc;

int krr_sketch_locate(krr_ctx* ctx, int64_t n_segments, const uint32_t* counts, const krr_sketch_params* sp,
                      const krr_percentile_params* params, krr_sketch_loc* out, void* stream);
/* out[s] = local samples in [loc[s].bin_lo, loc[s].bin_hi] (from this rank's own sketch). */
int krr_sketch_range_count(krr_ctx* ctx, int64_t n_segments, const uint32_t* counts, const krr_sketch_params* sp,
                           const krr_sketch_loc* loc, int64_t* out, void* stream);
/* Segment s's present samples with bin in [bin_lo, bin_hi], position order, to
 * out_values[out_offsets[s] ...]; out_count[s] (optional) = how many were written. */
int krr_sketch_collect(krr_ctx* ctx, const krr_series* series, const krr_sketch_params* sp,
                       const krr_sketch_loc* loc, const int64_t* out_offsets, double* out_values,
                       int64_t* out_count, void* stream);
/* collected: one segment per series (all ranks' lists, time order); out_flags adds
 * KRR_FLAG_CAPACITY if a list does not hold the located ranks. */
int krr_sketch_refine(krr_ctx* ctx, const krr_series* collected, const krr_sketch_loc* loc, double* out_value,
                      int64_t* out_count, uint32_t* out_flags, void* stream);

/* ---- Exact time-sharded percentiles in ONE HBM pass (config 5, window export) ----
 * A series too long for one GPU is time-sharded: rank r holds its r-th time slice.
 *   1. every rank: krr_window_export streams each local slice ONCE and keeps, in LDS,
 *      the exact contents of a key window that narrows around where the GLOBAL
 *      percentile's ranks are expected to fall (the slice's samples are read as a
 *      sample of the whole series: ext_slots = the other ranks' slots per series widen
 *      the window by the uncertainty they add).  Per series it writes a krr_window_hdr
 *      and the window's keys (order-preserving uint64 keys, -0 < +0) into a row of
 *      key_cap keys;
 *   2. the owner of a series receives every rank's header and row (RCCL all-to-all);
 *   3. krr_window_merge intersects the ranks' windows [max lo, min hi]; the headers'
 *      exact counts say whether the needed ranks lie inside it — then they are selected
 *      there, bit-identical to krr_segmented_percentile on the whole series — or not
 *      (a slice whose distribution differs from the series', e.g. a trend): then the
 *      series is flagged KRR_FLAG_WINDOW_MISS and counted in *miss_count, and the caller
 *      finishes it exactly (krr_amd.core.sketch: its slices regathered to the owner).
 * Nothing statistical is trusted: a hit is decided by exact counts. */
#define KRR_FLAG_WINDOW_MISS 16u  /* krr_window_merge: the needed ranks are not inside the
                                     ranks' common window (value NaN): finish it elsewhere */
#define KRR_WIN_FAIL 0x100u       /* krr_window_hdr.flags: no usable window (keys crowded the LDS) */
#define KRR_WIN_POINT 0x200u      /* the window is one key (lo == hi): cnt copies of it, no keys stored */

typedef struct {
    uint64_t lo, hi;   /* inclusive key window */
    int64_t below;     /* present samples of the slice with key < lo */
    int64_t n;         /* present samples of the slice (compact layout: every slot) */
    uint32_t cnt;      /* samples with key in [lo, hi]: the first cnt keys of the row */
    uint32_t flags;    /* KRR_WIN_FAIL, KRR_WIN_POINT, KRR_FLAG_NAN (compact layout) */
} krr_window_hdr;      /* 40 bytes */

/* Keys per row for slices of up to max_slice_len slots with ext_slots slots elsewhere
 * (host only; 0 for REF_INDEX or invalid arguments). */
int64_t krr_window_key_cap(int64_t max_slice_len, int64_t ext_slots, const krr_percentile_params* params);
/* hdr[S], keys[S * key_cap] (device).  SORTED_LOWER / LINEAR only. */
int krr_window_export(krr_ctx* ctx, const krr_series* slices, const krr_percentile_params* params,
                      int64_t ext_slots, int64_t key_cap, krr_window_hdr* hdr, uint64_t* keys, void* stream);
/* n_series series, each with n_slices slices in time order: slice j of series i has
 * header hdr[j * slice_stride + i] and keys keys[(j * slice_stride + i) * key_cap ...].
 * Writes out_value / out_count / out_flags[n_series]; *miss_count (device uint32, may
 * be NULL) is zeroed on the stream, then counts the KRR_FLAG_WINDOW_MISS series. */
int krr_window_merge(krr_ctx* ctx, int64_t n_series, int32_t n_slices, int64_t slice_stride,
                     const krr_window_hdr* hdr, const uint64_t* keys, int64_t key_cap,
                     const krr_percentile_params* params, double* out_value, int64_t* out_count,
                     uint32_t* out_flags, uint32_t* miss_count, void* stream);

/* Per segment: out_lt[s] = #present samples < values[s], out_le[s] = #<= values[s]. */
int krr_rank_of(krr_ctx* ctx, const krr_series* series, const double* values, int64_t* out_lt,
                int64_t* out_le, void* stream);

/* Per segment: out[s] = the k[s]-th present sample (0-based, position order; NaN
 * slots absent when gaps_are_nan), skipped when k[s] < 0.  The local step of the
 * exact time-sharded REF_INDEX (simple.py:36 over the concatenated slices). */
int krr_select_present(krr_ctx* ctx, const krr_series* series, const int64_t* k, double* out,
                       void* stream);

/* Where a selected value sits in its segment (the sample OBJECT the reference returns,
 * strategies/simple.py:29 `max(data_)` and :36 `data_[k]`, for inputs whose Decimals the
 * float64 values do not reproduce character for character).  Per segment s with
 * rank[s] >= -1: out_lt[s] = #samples < values[s], out_eq[s] = #samples == values[s]
 * (float ==: -0 == +0; NaN equals nothing), out_pos[s] = slot offset (from the segment
 * start) of the j-th sample equal to values[s] in position order, j = rank[s] - out_lt[s]
 * (the element sorted(X)[rank] of a stable sort) or j = 0 when rank[s] == -1 (the first
 * maximal element max() keeps); -1 when there is no such sample.  rank[s] < -1: segment
 * skipped, its outputs untouched.  Device pointers, n_segments entries each. */
int krr_locate(krr_ctx* ctx, const krr_series* series, const double* values, const int64_t* rank, int64_t* out_lt,
               int64_t* out_eq, int64_t* out_pos, void* stream);

/* Synthetic week-long series (bench/test data), generated on the device from a
 * counter-based hash so that no host packing or PCIe is involved.
 * kind 0 = CPU cores ~ Gamma(k=2, theta=0.05); kind 1 = memory bytes
 * floor(Normal(2e8, 2e7)).  Segment s holds pods of pod_len slots (the last pod
 * takes the remainder); with gaps != 0, each pod gets a late start with prob.
 * 0.3 (>= 1440 samples kept), and gap runs in blocks of 30 slots with a per-pod
 * gap fraction ~ U(0, 0.2); gap slots are NaN. */
int krr_synth_fill(krr_ctx* ctx, double* values, const int64_t* offsets, int64_t n_segments,
                   uint64_t seed, int32_t kind, int64_t pod_len, int32_t gaps, void* stream);

/* Same, for the time window [t0, t0 + len) of series of total_len slots: slot i
 * of segment s holds global time index t0 + i, so slices generated on different
 * ranks concatenate to the series krr_synth_fill would generate whole. */
int krr_synth_fill_window(krr_ctx* ctx, double* values, const int64_t* offsets, int64_t n_segments,
                          uint64_t seed, int32_t kind, int64_t pod_len, int32_t gaps, int64_t t0,
                          int64_t total_len, void* stream);

/* Same, with segment s of this call being GLOBAL segment seg_base + s of the fleet:
 * a rank that owns objects [seg_base, seg_base + n_segments) generates exactly the
 * series a single GPU generates for them (krr_synth_fill == seg_base 0). */
int krr_synth_fill_global(krr_ctx* ctx, double* values, const int64_t* offsets, int64_t n_segments,
                          uint64_t seed, int32_t kind, int64_t pod_len, int32_t gaps, int64_t seg_base,
                          int64_t t0, int64_t total_len, void* stream);

/* ---- Device packer: Prometheus query_range bodies -> CSR in HBM (round 3) ----
 * Replaces, for bodies already copied to HBM, the host packer krr_pack_parse
 * (include/krr_pack.h), i.e. the reference's per-pod
 *   [Decimal(value) for _, value in pod_result[0]["values"]] + the empty-pod drop
 * of PrometheusLoader.gather_data, robusta_krr/core/integrations/prometheus.py:147-155.
 * One wave per body.  A body whose bytes lie outside the canonical query_range form
 * Prometheus writes (escapes in keys or values, whitespace inside a value string,
 * spellings of NaN/Inf other than "NaN"/"Inf", more than 19 significant digits,
 * status != "success", malformed JSON) is NOT an error here: its status is
 * KRR_JSON_HOST and the caller parses that batch with krr_pack_parse, which returns
 * the host packer's result or error.  Whatever this packer accepts it parses to the
 * bits krr_pack_parse produces.
 *
 * Two steps on `stream`:
 *   krr_json_parse    every body of [first, first + n): status[b], counts[b] (samples
 *                     kept; 0 unless KRR_JSON_OK), values (and timestamps) written to
 *                     scratch slot (body_offsets[b] / 8) + i;
 *   krr_json_compact  each KRR_JSON_OK body's run to values[out_pos[b] ..) — out_pos
 *                     the exclusive prefix sum of counts (the CSR of the caller's
 *                     objects follows from the counts, bodies in fleet order).
 * Buffers: bodies 16-byte aligned with 128 readable bytes past the last body;
 * scratch_values / scratch_ts hold body_offsets[n_bodies] / 8 + 1 doubles. */
#define KRR_JSON_OK 0        /* parsed: counts[b] samples */
#define KRR_JSON_DROPPED 1   /* data.result is empty: the pod is dropped (prometheus.py:154) */
#define KRR_JSON_HOST 2      /* outside the device grammar: parse the batch with krr_pack_parse */

typedef struct krr_json_bodies {
    const char* bodies;           /* device: the response bodies back to back */
    const int64_t* body_offsets;  /* device: [n_bodies + 1] byte offsets, body_offsets[0] == 0 */
    int64_t n_bodies;
    int64_t total_bytes;          /* body_offsets[n_bodies] (host copy) */
} krr_json_bodies;

int krr_json_parse(krr_ctx* ctx, const krr_json_bodies* b, int64_t first, int64_t n, int32_t want_timestamps,
                   double* scratch_values, double* scratch_ts, int64_t* counts, int32_t* status, void* stream);
int krr_json_compact(krr_ctx* ctx, const krr_json_bodies* b, const double* scratch_values,
                     const double* scratch_ts, const int64_t* counts, const int32_t* status,
                     const int64_t* out_pos, double* values, double* timestamps, void* stream);

/* n host -> device copies enqueued on `stream` in order (dst[i] <- src[i], bytes[i] bytes;
 * src page-locked for an asynchronous copy): the device packer's staged runs and body
 * offsets, one call per chunk instead of one runtime call per run from Python. */
int krr_copy_h2d_batch(krr_ctx* ctx, int64_t n, void* const* dst, const void* const* src, const int64_t* bytes,
                       void* stream);

/* Grouped bodies (`sum by (pod) (...)`, one series per pod: the host packer's
 * krr_pack_parse_grouped, include/krr_pack.h), one wave per SERIES:
 *   krr_json_find_series    every `[{"metric":` / `,{"metric":` starting in [begin, end) whose
 *                           11 bytes lie below `limit` (the bytes already copied: a caller
 *                           searches each chunk as it lands, the chunk's last 16 bytes
 *                           with the next one): the absolute offset of its '{' appended at
 *                           candidates[*n_candidates ..]
 *                           (device counter, zeroed by the caller; any order; the count
 *                           may exceed cap, then only cap are stored);
 *   krr_json_parse_segments one series object per candidate (sorted starts, body_of[j] its
 *                           body): segments[j] = 7 int64 {start, end (one past its '}', -1
 *                           when it is not a series object), label value offset (-1: none),
 *                           label length, scratch slot of its values (array offset / 8),
 *                           count, ok}.
 * The host then chains the segments from each body's envelope (krr_pack_route_grouped,
 * include/krr_pack.h); a body whose series do not chain goes to the host packer.
 * Bodies need 128 readable bytes past the last one. */
int krr_json_find_series(krr_ctx* ctx, const krr_json_bodies* b, int64_t begin, int64_t end, int64_t limit,
                         int64_t* candidates, int64_t cap, uint64_t* n_candidates, void* stream);
int krr_json_parse_segments(krr_ctx* ctx, const krr_json_bodies* b, const int64_t* starts, const int64_t* body_of,
                            int64_t n, const char* label, int32_t want_timestamps, double* scratch_values,
                            double* scratch_ts, int64_t* segments, void* stream);
/* krr_json_parse_segments with each series' values array parsed by several waves (round 6):
 * the series' wave finds the array's end and cuts it into 16-KiB parts, then one wave per part
 * parses its elements (same segments, scratch values and validation).  workspace: device
 * int64 [workspace_words] = 1 (part counter) + n (array ends) + 6 per part; a series whose
 * parts find no room is reported not ok (its body goes to the host packer), so
 * (bytes of the candidates' bodies) / 16384 + 2 n parts always suffice.  Replaces nothing in
 * the reference: the host-side equivalent is krr_pack_parse_grouped (include/krr_pack.h). */
int krr_json_parse_segments_split(krr_ctx* ctx, const krr_json_bodies* b, const int64_t* starts,
                                  const int64_t* body_of, int64_t n, const char* label, int32_t want_timestamps,
                                  double* scratch_values, double* scratch_ts, int64_t* segments, int64_t* workspace,
                                  int64_t workspace_words, void* stream);
/* values[dst[j] ..) = scratch_values[src[j] ..), count[j] values (count < 0: none); the same
 * for timestamps when both pointers are given. */
int krr_json_gather(krr_ctx* ctx, int64_t n_items, const int64_t* src, const int64_t* count, const int64_t* dst,
                    const double* scratch_values, const double* scratch_ts, double* values, double* timestamps,
                    void* stream);

#ifdef __cplusplus
}
#endif

#endif /* KRR_AMD_H */
