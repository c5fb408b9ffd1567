// poly.hpp — LDS-staged polyphase FIR machinery for gfx950 (device side).
//
// A decimate-by-M FIR with K <= M*Q real taps g[k] evaluated only at the kept
// outputs:  d[j] = sum_k g[k] * x[M*j - k]   (k = M*q + c).
// Polyphase split: u_c[i] = x[M*i - c]  =>  d[j] = sum_c sum_q g[M*q + c] * u_c[j - q].
//
// One sub-tile produces T consecutive outputs d[J .. J+T). Its M*(T+Q) input
// samples (origin P_org = M*(J - Q)) are staged once into LDS, de-interleaved by
// phase: U[c][i'] with i' = i - J + Q. Each lane then owns R = T/NT consecutive
// outputs and, per phase, reads a (R+Q)-sample window with ds_read_b128 (two cf32
// per read) and accumulates with packed FMAs (I/Q in one v_pk_fma_f32, the real
// tap broadcast from an SGPR). Row pitch LR is even (16-B aligned reads) and
// LR = 2 (mod 16) so the phase-scattered ds_write_b64 stores spread over banks;
// the lane stride of the reads (R = 2 cf32 = 16 B) makes the b128 reads of a
// 16-lane group hit 16 distinct 4-bank slots (conflict-free).
#pragma once
#include "hip_common.hpp"

namespace orion {

__device__ __forceinline__ float fmav(float g, float x, float a) { return __builtin_fmaf(g, x, a); }
__device__ __forceinline__ f2 fmav(float g, f2 x, f2 a) { return fma2(splat2(g), x, a); }

template <int M, int Q, int T, int NT>
struct Poly {
  static_assert((M & (M - 1)) == 0, "M must be a power of two on this path");
  static constexpr int R = T / NT;
  static_assert(R * NT == T && (R % 2) == 0, "two (or an even number of) outputs per lane");
  static constexpr int NS = M * (T + Q);                  // staged samples per sub-tile
  static constexpr int LR = ((T + Q + 1 + 15) / 16) * 16 + 2;
  static constexpr int LDS_F2 = M * LR;                   // cf32 slots of LDS
  static constexpr int W = R + Q;                         // window per lane and phase
  static_assert((W % 2) == 0, "window read as cf32 pairs");

  // Staged sample p' (0 <= p' < NS) -> LDS slot.
  __device__ __forceinline__ static int slot(int p) {
    const int c = (-p) & (M - 1);
    const int i = (p + c) / M;
    return c * LR + i;
  }

  // Accumulate the lane's R outputs. gp(c, q) returns tap g[M*q + c]; taps are
  // stored phase-major (gp row c = 16/32 consecutive floats) so that each phase
  // iteration issues one scalar s_load_dwordx16 and keeps SGPR pressure flat.
  // The phase loop is deliberately not unrolled (kernarg hoisting of every tap
  // would otherwise spill SGPRs).
  template <class TapFn>
  __device__ __forceinline__ static void compute(const f2* __restrict__ U, int lane, TapFn gp,
                                                 f2 (&acc)[R]) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = f2{0.0f, 0.0f};
#pragma unroll 1
    for (int c = 0; c < M; ++c) {
      const f4* row = reinterpret_cast<const f4*>(U + c * LR + R * lane);
#pragma unroll
      for (int h = 0; h < W / 2; ++h) {
        const f4 v = row[h];
        const f2 w0 = f2{v.x, v.y}, w1 = f2{v.z, v.w};
        // window index m -> output r uses tap q = r + Q - m
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int q0 = r + Q - 2 * h, q1 = r + Q - 2 * h - 1;
          if (q0 >= 0 && q0 < Q) acc[r] = fma2(splat2(gp(c, q0)), w0, acc[r]);
          if (q1 >= 0 && q1 < Q) acc[r] = fma2(splat2(gp(c, q1)), w1, acc[r]);
        }
      }
    }
  }
};

// Two consecutive outputs of a K-tap FIR, taps in blocks of 16 (one scalar
// s_load_dwordx16 per block; the block loop is rolled to keep SGPRs flat):
//   acc_r += sum_{k < KP} g(k) * X[e + r - k],  r = 0, 1,  e even.
// rd(i) returns the aligned element pair (X[i], X[i+1]) for even i.
template <int KP, class V, class Rd, class Tap>
__device__ __forceinline__ void fir2_blocked(Rd rd, long long e, Tap g, V& acc0, V& acc1) {
  static_assert(KP % 16 == 0, "taps padded to 16");
#pragma unroll 1
  for (int kb = 0; kb < KP / 16; ++kb) {
    const long long e0 = e - 16 * kb - 16;
#pragma unroll
    for (int h = 0; h < 9; ++h) {
      V w[2];
      rd(e0 + 2 * h, w[0], w[1]);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int m = 2 * h + u;  // element e0 + m; output r uses k = 16*kb + 16 + r - m
        const int k0 = 16 - m, k1 = 17 - m;
        if (k0 >= 0 && k0 < 16) acc0 = fmav(g(16 * kb + k0), w[u], acc0);
        if (k1 >= 0 && k1 < 16) acc1 = fmav(g(16 * kb + k1), w[u], acc1);
      }
    }
  }
}

// Load cf32 sample P of a stream whose samples [0, n) live at x, whose
// samples [-hist_len, 0) live at hist[hist_len + P], and which is zero elsewhere.
__device__ __forceinline__ f2 load_hist(const f2* __restrict__ x, long long n,
                                        const f2* __restrict__ hist, int hist_len, long long P) {
  if (P >= 0) return P < n ? x[P] : f2{0.0f, 0.0f};
  if (P >= -hist_len) return hist[hist_len + P];
  return f2{0.0f, 0.0f};
}

// Pair load (P even): one 16-B load when fully inside [0, n) and 16-B aligned.
template <bool A16>
__device__ __forceinline__ void load_pair(const f2* __restrict__ x, long long n,
                                          const f2* __restrict__ hist, int hist_len, long long P,
                                          f2& v0, f2& v1) {
  if (P >= 0 && P + 1 < n) {
    if constexpr (A16) {
      const f4 v = *reinterpret_cast<const f4*>(x + P);
      v0 = f2{v.x, v.y};
      v1 = f2{v.z, v.w};
    } else {
      v0 = x[P];
      v1 = x[P + 1];
    }
  } else {
    v0 = load_hist(x, n, hist, hist_len, P);
    v1 = load_hist(x, n, hist, hist_len, P + 1);
  }
}

}  // namespace orion
