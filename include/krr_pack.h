/*
 * krr_pack.h — host-side C ABI of the native Prometheus query_range packer.
 *
 * Replaces the reference's per-pod response handling in
 *   PrometheusLoader.gather_data  robusta_krr/core/integrations/prometheus.py:108-155
 * which, for every pod of an object, takes custom_query_range(...)'s result
 * (prometheus_api_client 0.5.3: response.json()["data"]["result"]), drops a pod
 * whose result list is empty, keeps ONLY the first series' "values", discards the
 * timestamps and parses each value string with Decimal() (prometheus.py:147-155).
 * Here whole HTTP response bodies go in, in parallel, and one CSR float64 buffer
 * per resource comes out — the layout libkrr_amd's kernels read (krr_amd.h).
 *
 * Value strings are Prometheus' shortest round-trip float formatting ("0.0123",
 * "1e-05", "NaN", "+Inf", "-Inf"); each is parsed to the float64 it denotes
 * (correctly rounded, std::from_chars), so the host's exact-decimal rounding
 * sees Decimal(repr(x)) == Decimal(string) for every such string.
 *
 * Ownership: krr_pack_parse returns an opaque result the caller frees with
 * krr_pack_free; krr_pack_copy fills caller-owned buffers.  No function throws.
 */
#ifndef KRR_PACK_H
#define KRR_PACK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KRR_PACK_ABI_VERSION 1

typedef enum {
    KRR_PACK_OK = 0,
    KRR_PACK_E_INVALID = -1,   /* bad argument */
    KRR_PACK_E_PARSE = -2,     /* a body is not a query_range JSON response (see krr_pack_error) */
    KRR_PACK_E_STATUS = -3,    /* a body's "status" is not "success" */
    KRR_PACK_E_VALUE = -4      /* a sample value string is not a number */
} krr_pack_status;

typedef struct krr_pack krr_pack;

int krr_pack_abi_version(void);

/* Parse n_bodies response bodies (body b = bodies[b][0 .. body_lens[b])) on up to
 * `threads` host threads (<= 0: all hardware threads).  Body b is one pod of object
 * obj_of_body[b]; obj_of_body is non-decreasing (objects in fleet order, each
 * object's pods in K8sObjectData.pods order), values in [0, n_objects).
 * want_timestamps != 0 keeps each sample's timestamp (seconds) as well.
 * On success *out holds the result (free with krr_pack_free); on a parse error
 * *out still holds a result whose krr_pack_error() names the first bad body. */
int krr_pack_parse(const char* const* bodies, const int64_t* body_lens, int64_t n_bodies,
                   const int64_t* obj_of_body, int64_t n_objects, int32_t want_timestamps,
                   int32_t threads, krr_pack** out);

/* Total samples kept (over all objects). */
int64_t krr_pack_n_values(const krr_pack* p);
/* Longest object segment (planning hint for the kernels' max_segment_len). */
int64_t krr_pack_max_len(const krr_pack* p);

/* Fill caller buffers: values[n_values]; offsets[n_objects + 1] (segment s =
 * object s's kept pods concatenated); optional (NULL to skip): timestamps[n_values]
 * (needs want_timestamps), pod_counts[n_bodies] (samples kept per body, -1 for a
 * dropped pod: empty result list). */
int krr_pack_copy(const krr_pack* p, double* values, int64_t* offsets, double* timestamps,
                  int64_t* pod_counts, int32_t threads);

/* First error ("" when none). */
const char* krr_pack_error(const krr_pack* p);

void krr_pack_free(krr_pack* p);

/* ---- Grouped responses (fleet-level query batching) ----
 * One `sum by (pod) (...)` range query per (namespace, container) replaces one
 * `sum(...{pod="..."})` query per pod (prometheus.py:118-143); its response holds
 * one series per pod.  krr_pack_parse_series splits such a body into its series,
 * each tagged with its metric's `label` value, for the caller to route to
 * (object, pod) slots in K8sObjectData.pods order. */
typedef struct krr_series_set krr_series_set;

int krr_pack_parse_series(const char* body, int64_t len, const char* label, int32_t want_timestamps,
                          krr_series_set** out);
int64_t krr_series_count(const krr_series_set* h);
/* NUL-terminated label value of series i; *len = its byte length, or -1 if the
 * series has no such label. */
const char* krr_series_label(const krr_series_set* h, int64_t i, int64_t* len);
int64_t krr_series_len(const krr_series_set* h, int64_t i);
int krr_series_copy(const krr_series_set* h, int64_t i, double* values, double* timestamps);
const char* krr_series_error(const krr_series_set* h);
void krr_series_free(krr_series_set* h);

/* The whole fleet at once: n_bodies grouped response bodies in, one krr_pack out
 * (read it with krr_pack_n_values / krr_pack_max_len / krr_pack_copy, exactly as
 * krr_pack_parse's).  Slot s is one (object, pod) pair in fleet order: its pod name
 * is slot_names[slot_name_offsets[s] .. slot_name_offsets[s+1]), its series is the
 * first one in body slot_body[s] whose metric[label] equals that name (none: the
 * pod is dropped, pod_counts[s] = -1, as the reference drops an empty result), and
 * obj_of_slot is non-decreasing in [0, n_objects).  krr_pack_copy's pod_counts is
 * then indexed by slot. */
int krr_pack_parse_grouped(const char* const* bodies, const int64_t* body_lens, int64_t n_bodies, const char* label,
                           const int64_t* slot_body, const char* slot_names, const int64_t* slot_name_offsets,
                           const int64_t* obj_of_slot, int64_t n_slots, int64_t n_objects, int32_t want_timestamps,
                           int32_t threads, krr_pack** out);

/* Staging for the device packer (include/krr_amd.h krr_json_parse): body b's bytes to
 * dst[dst_offsets[b] - dst_offsets[0] ..) for b in [0, n_bodies), on up to `threads`
 * host threads (dst typically page-locked memory the H2D copy reads by DMA). */
int krr_pack_concat(const char* const* bodies, const int64_t* body_lens, int64_t n_bodies,
                    const int64_t* dst_offsets, char* dst, int32_t threads);

/* The same staging with each sample timestamp cut to its first digit (krr_amd/csrc/krr_strip.h:
 * `[1700000000.25,"0.3"]` -> `[1,"0.3"]`; the reference drops timestamps,
 * robusta_krr/core/integrations/prometheus.py:152).  A body outside the strippable form
 * (whitespace or a backslash in its values array, a timestamp other than
 * (0|[1-9][0-9]*)(.[0-9]+)?, a CPU without AVX-512 VBMI2) is copied unchanged.  Bodies are cut
 * into at most `max_runs` contiguous runs (by bytes); run r = bodies [run_first[r],
 * run_first[r + 1]) is written back to back from dst[dst_offsets[run_first[r]] - dst_offsets[0]],
 * inside the run's own unstripped extent.  new_lens[b] = bytes written for body b; *n_runs = the
 * runs used (run_first holds n_runs + 1 entries, run_first[n_runs] == n_bodies).
 * Neither the device parser nor the host packer reads a timestamp's value without
 * want_timestamps, so a stripped body packs to the same CSR as the original. */
int krr_pack_concat_strip(const char* const* bodies, const int64_t* body_lens, int64_t n_bodies,
                          const int64_t* dst_offsets, char* dst, int32_t threads, int32_t max_runs,
                          int64_t* new_lens, int64_t* run_first, int32_t* n_runs);

/* The same stripped staging in PIECES that may split a large body (grouped `sum by (pod)` bodies
 * of ~100 MB, which one thread would strip alone): bodies of fewer than 2P bytes (P = total /
 * max_pieces) go in runs of whole bodies as above; a larger one is cut near every P bytes at a
 * sample's '[' after a value string (`"],[` whose quote closes a string, found from the quote
 * parity counted in parallel; a strippable body has no backslash), where no token spans the cut,
 * so its pieces strip apart to exactly what the whole-body copy writes.  Piece j starts at byte
 * piece_start[j] of the unstripped layout (dst_offsets coordinates; piece_start[n_pieces] = the
 * end) and its piece_out[j] stripped bytes are written from dst[piece_start[j] - dst_offsets[0]]
 * on; the pieces concatenated in order are the stripped bodies back to back.  new_lens[b] = the
 * stripped bytes of body b.  A body with an unstrippable piece is copied unchanged.  piece_start
 * needs 2 n_bodies + max_pieces + 1 entries, piece_out 2 n_bodies + max_pieces. */
int krr_pack_concat_strip_pieces(const char* const* bodies, const int64_t* body_lens, int64_t n_bodies,
                                 const int64_t* dst_offsets, char* dst, int32_t threads, int32_t max_pieces,
                                 int64_t* new_lens, int64_t* piece_start, int64_t* piece_out, int32_t* n_pieces);

/* One body stripped as above into out (body_len bytes of room): the bytes written, or -1
 * when it is not strippable.  (Tests and probes.) */
int64_t krr_pack_strip_body(const char* body, int64_t body_len, char* out);

/* Routing for the device packer's grouped bodies (include/krr_amd.h krr_json_find_series /
 * krr_json_parse_segments).  `bodies` is the staged host copy of the device buffer (same
 * offsets).  Per body: the envelope is walked up to data.result's first series, the
 * device's segments (n_segments x 7 int64 {start, end, label offset, label length,
 * scratch slot, count, ok}, sorted by start) must chain from there, one series after
 * the next, and the envelope's tail is walked (krr_json_parse.h chain_grouped);
 * body_ok[b] = 0 when they do not (the caller parses the batch with
 * krr_pack_parse_grouped).  Slot s (body slot_body[s], pod name slot_names[
 * slot_name_offsets[s] .. slot_name_offsets[s+1])) takes the FIRST chained series of its
 * body whose `label` equals the name, as krr_pack_parse_grouped does: slot_src[s] /
 * slot_count[s] = its scratch slot and count, or -1 / -1 (dropped). */
int krr_pack_route_grouped(const char* bodies, const int64_t* body_offsets, int64_t n_bodies, const char* label,
                           const int64_t* segments, int64_t n_segments, const int64_t* slot_body,
                           const char* slot_names, const int64_t* slot_name_offsets, int64_t n_slots,
                           int64_t* slot_src, int64_t* slot_count, int32_t* body_ok, int32_t threads);

/* The same over a staged copy whose bytes do not sit at their device offsets: the staged
 * pieces of krr_pack_concat_strip(_pieces) — piece j holds device positions [piece_dev[j],
 * piece_dev[j + 1]) (ascending; the last one to the end), the byte at device position p of it
 * at bodies[p + piece_shift[j]].  Pieces cut a body only inside values arrays, so the envelope,
 * the bytes between series and every label sit inside one piece each. */
int krr_pack_route_grouped_pieces(const char* bodies, const int64_t* body_offsets, int64_t n_bodies,
                                  const int64_t* piece_dev, const int64_t* piece_shift, int64_t n_pieces,
                                  const char* label, const int64_t* segments, int64_t n_segments,
                                  const int64_t* slot_body, const char* slot_names,
                                  const int64_t* slot_name_offsets, int64_t n_slots, int64_t* slot_src,
                                  int64_t* slot_count, int32_t* body_ok, int32_t threads);

#ifdef __cplusplus
}
#endif

#endif /* KRR_PACK_H */
