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

#ifdef __cplusplus
}
#endif

#endif /* KRR_PACK_H */
