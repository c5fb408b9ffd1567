/* A plain C11 consumer of the drop-in boundary (include/orion_sdr_amd.h), the way a
 * non-Python caller binds the library: no torch, no C++, only the header and the
 * shared library. It drives the reference's Block contract (core.rs:12-22) on host
 * buffers: a WbfmChain (docs/demodulate.md:128-133) built from the C2 design, fed
 * in ragged streaming calls, and checks the audio against the CPU oracle
 * (oracle/orion_oracle.c, TEST INFRASTRUCTURE: the checker, never the thing
 * measured) streamed in the same calls.
 *
 *   wbfm_c_consumer [n]     exit 0: parity within 1e-5 nrmse; 1: parity failed;
 *                           2: the library reported an error (no device: it fails
 *                              loudly, there is no CPU fallback).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "orion_oracle.h"
#include "orion_sdr_amd.h"

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? (size_t)strtoull(argv[1], NULL, 10) : ((size_t)1 << 20);
  const size_t chunk = 3 * ((size_t)1 << 16) + 8; /* a multiple of m = 8, ragged against n */
  const double fs = 10e6;
  float* a = malloc(n * sizeof(float));
  oc32* x = malloc(n * sizeof(oc32));
  const size_t cap = n / 8 + 1;
  float* y = malloc(cap * sizeof(float));
  float* yref = malloc(cap * sizeof(float));
  if (!a || !x || !y || !yref) return 2;
  /* SURVEY §8(d) C2 shape: 0.5 sin(2 pi 1k t) + 0.3 sin(2 pi 7k t), FM at 75 kHz
   * deviation on a +1.5 MHz carrier (the oracle's FmPhaseAccumMod), AWGN P = 0.0025 */
  for (size_t i = 0; i < n; ++i) {
    const double t = (double)i / fs;
    a[i] = (float)(0.5 * sin(2.0 * M_PI * 1000.0 * t) + 0.3 * sin(2.0 * M_PI * 7000.0 * t));
  }
  o_fm_mod mod;
  o_fm_mod_init(&mod, (float)fs, 75e3f, 1.5e6f);
  (void)o_fm_mod_process(&mod, a, x, n);
  o_add_awgn(x, n, 0.0025f, 0x12345678ABCDEF00ull);

  const orion_wbfm_params p = {(float)fs, 1.5e6f, 200e3f, 79e3f, 75e3f, 15e3f, 15e3f, 10e3f, 8};
  orion_block* b = orion_wbfm_chain_new(&p);
  if (!b) {
    fprintf(stderr, "orion_wbfm_chain_new: %s\n", orion_last_error());
    return 2;
  }
  printf("library %s, block %s, in type %d, out type %d\n", orion_version(), orion_block_name(b),
         orion_block_in_type(b), orion_block_out_type(b));
  size_t written = 0, calls = 0;
  for (size_t off = 0; off < n; off += chunk, ++calls) {
    const size_t len = n - off < chunk ? n - off : chunk;
    orion_work_report wr = {0, 0};
    const int rc = orion_block_process(b, x + off, len, y + written, cap - written, &wr);
    if (rc != ORION_OK || wr.in_read != len) {
      fprintf(stderr, "orion_block_process: rc %d in_read %zu of %zu: %s\n", rc, wr.in_read, len,
              orion_last_error());
      orion_block_free(b);
      return 2;
    }
    written += wr.out_written;
  }
  orion_block_free(b);

  const o_wbfm_params q = {(float)fs, 1.5e6f, 200e3f, 79e3f, 75e3f, 15e3f, 15e3f, 10e3f, 8};
  const size_t nref = o_run_wbfm(&q, x, n, yref, cap, chunk);
  double num = 0.0, den = 0.0;
  for (size_t i = 0; i < nref && i < written; ++i) {
    const double d = (double)y[i] - (double)yref[i];
    num += d * d;
    den += (double)yref[i] * (double)yref[i];
  }
  const double nrmse = den > 0.0 ? sqrt(num / den) : INFINITY;
  printf("[parity] C consumer: %zu samples in %zu host calls -> %zu audio (oracle %zu), nrmse %.3e (tol 1e-5)\n",
         n, calls, written, nref, nrmse);
  free(a);
  free(x);
  free(y);
  free(yref);
  return (written == nref && nrmse <= 1e-5) ? 0 : 1;
}
