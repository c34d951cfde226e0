/*
 * ddpca_probe.h -- C ABI of libddpca_probe.so: measurement probes beside the product library
 * (no reference counterpart).  bench.py and profiles/ load it; nothing in libddpca_amd.so does.
 * Error codes and ddpca_last_error() as in ddpca_amd.h (the probe library links libddpca_amd.so).
 */
#ifndef DDPCA_PROBE_H
#define DDPCA_PROBE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* SURVEY §8 d3's measured STREAM ceiling: a STREAM copy and a STREAM read of `bytes` per buffer
 * (>= 64 MiB; use >> the 256 MiB Infinity Cache), 16 B per lane, non-temporal, best of three
 * batches of `reps` launches on a stream of its own.
 * out4 = [copy GB/s (bytes read + written), read GB/s, copy ms, read ms]. */
int ddpca_stream_ceiling(int device, int64_t bytes, int reps, double* out4);
/* DESIGN §8, the persistent below-fine V-cycle: `phases` dependent passes over n doubles, each
 * reading what other workgroups wrote in the previous pass, run as one hipGraph of `phases`
 * launches and as one persistent launch with a grid barrier between passes, `blocks` workgroups of
 * 256 each way.  pin = 0: the persistent workgroups spread over the 8 XCDs (blocks <= CUs);
 * pin = 1: 8 x blocks workgroups launched, only those with id % 8 == 0 work (one XCD under the
 * round-robin dispatch; blocks <= CUs / 8), the others exit at once.  The barrier is the release /
 * relaxed-poll / acquire counter form (agent scope: co-location gives no visibility).
 * out4 = [graph us per pass, persistent us per pass, max |difference| of the two results, 1 if a
 * persistent workgroup timed out waiting]. */
int ddpca_probe_grid_barrier(int device, int64_t n, int phases, int blocks, int pin, double* out4);

#ifdef __cplusplus
}
#endif

#endif  // DDPCA_PROBE_H
