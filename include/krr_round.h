/*
 * krr_round.h — host C ABI of the batched exact-decimal post-processor.
 *
 * Replaces, for every object at once, the reference's per-object Decimal work
 * after the kernels:
 *   memory proposal  max(X) * Decimal(1 + b/100)      strategies/simple.py:24-29
 *   Runner._round_value (ceil to 1m CPU / 1M memory)   core/runner.py:57-77
 *   Runner.__get_resource_minimal (clamp)              core/runner.py:49-55
 * in the reference's decimal context (prec 28, ROUND_HALF_EVEN).  The float64
 * sample the GPU selected is first turned into the Decimal the reference parsed
 * from Prometheus' string (shortest round-trip digits, positional; the
 * prom_decimal rule), then every step is exact decimal arithmetic on digit
 * strings.  Each result is written as Python's str(Decimal) of the reference's
 * Decimal — same digits AND exponent (e.g. "2.1E+7" vs "21000000"), so
 * Decimal(s) reproduces the reference's object exactly.
 *
 * Objects this path does not cover (a non-finite value, a NaN sample flag,
 * > 28-digit intermediates) get a status bit, and the caller applies the
 * Python restatement (krr_amd/core/rounding.py) to those alone.
 */
#ifndef KRR_ROUND_H
#define KRR_ROUND_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    const char* mem_buffer;   /* str(Decimal(1 + b/100)) as the strategy computes it (e.g. "1.05") */
    const char* cpu_minimal;  /* str() of Runner.__get_resource_minimal(CPU), e.g. "0.005000000000000000104083408559" */
    const char* mem_minimal;  /* str() of the memory minimal, e.g. "10000000" */
    int32_t fast_path;        /* 1: 128-bit integer arithmetic where the operands fit (same results);
                                 0: digit strings throughout (the reference restatement, for tests) */
    int32_t reserved;
} krr_round_params;

#define KRR_ROUND_CPU_FALLBACK 1u  /* cpu_out[i] not written: use the Python path */
#define KRR_ROUND_MEM_FALLBACK 2u  /* mem_out[i] not written: use the Python path */

/* Per object i (flags are the kernels' KRR_FLAG_* words):
 *   cpu_out + i*width: str(round_value(prom_decimal(cpu_value[i]), CPU))   ("NaN" when empty)
 *   mem_out + i*width: str(round_value(prom_decimal(mem_value[i]) * buffer, Memory))
 * width >= 64.  status[i] = KRR_ROUND_* bits.  threads <= 0: all hardware threads.
 * Returns 0, or -1 for bad arguments (unparsable parameter strings included). */
int krr_round_simple(int64_t n, const double* cpu_value, const uint32_t* cpu_flags, const double* mem_value,
                     const uint32_t* mem_flags, const krr_round_params* params, char* cpu_out, char* mem_out,
                     int32_t width, uint8_t* status, int32_t threads);

#ifdef __cplusplus
}
#endif

#endif /* KRR_ROUND_H */
