// k_wbfm.hip — the WBFM demodulation chain on gfx950 (the north-star path).
//
// Reference composition (docs/demodulate.md:128-133, SURVEY §3 stack 2):
//   Rotator(-f_off).rotate_block (dsp/rotator.rs:74-85)
//   -> FirDecimator(fs, 8, ...)  (dsp/decim.rs:44-76; kept outputs only here)
//   -> FmQuadratureDemod         (demodulate/fm.rs:45-77: discriminator + LpCascade)
//   -> FirLowpass                (dsp/fir.rs:47-66, the audio filter).
//
// Building blocks (one 64-lane wave each, no workgroup barriers):
//   front tile (fu_tile)  — 1024 cf32 inputs -> 128 decimated outputs: the tile's
//     inputs were prefetched two tiles ahead (16-B nontemporal loads into
//     registers), are NCO-mixed with per-lane phasors and scattered into an
//     8-row polyphase LDS image (17-column halo carried from the previous tile),
//     the 127-tap polyphase FIR runs at the kept outputs (two per lane, packed
//     FMA, taps from SGPRs), the tile's common phasor multiplies them, and the
//     discriminator (atan2_approx op for op) writes 128 phi.
//   sub-range IIR — LpCascade over 1024 phi: a zero-state packed pass over two
//     halves, f64 Kogge-Stone scans, then the reference's f32 TDF-II recurrence
//     -> the audio FIR's pair image (f[j], f[j+512]); audio FIR = 125 taps in
//     8 blocks of 16, one v_pk_fma_f32 per tap for both halves.
// Kernels:
//   k_wbfm_seg2  (default) — one round of waves; each walks a segment of
//     1024-output sub-ranges, the IIR between tiles and the audio FIR spread
//     over the next sub-range's tiles; a segment's first sub-range is handed to
//     its predecessor (see the comment at the kernel).
//   k_wbfm_ws    — wave-specialised segments: 8 streaming waves and 4 back
//     waves per CU, phi through an LDS ring (ORION_WBFM_SPECIALIZED; timing
//     experiment, slower than k_wbfm_seg2: see DESIGN.md §5).
//   k_wbfm_seg   — the same segments with each sub-range's whole back run at
//     once and the first sub-range deferred to the end (ORION_WBFM_SEGMENTED_V1).
//   k_wbfm_fused — one wave per 2048-output range, two rounds of waves, zero-
//     state IIR hand-off between neighbouring ranges (ORION_WBFM_RANGES).
//   k_wbfm_front2 + k_wbfm_back — the two-kernel path (phi through HBM, a
//     510-sample IIR warm-up per 2048 outputs): any IIR design, used when the
//     LpCascade decays too slowly for the hand-offs above (ORION_WBFM_SPLIT).
// The first tile / sub-range of each channel starts from the exact state carried
// from the previous call (last decimated sample, 128 raw inputs, IIR state, last
// 128 IIR outputs), so k calls equal one call on the concatenation.
#include <algorithm>
#include <cstdlib>

#include "iir.hpp"
#include "kernels.hpp"
#include "poly.hpp"

namespace orion {
namespace {

constexpr int NT = 256;
constexpr int T = kWbfmT;
constexpr int M = kWbfmM;
constexpr int Q = kWbfmQ;
using PW = Poly<M, Q, T, NT>;
static_assert(PW::NS == kWbfmNS, "staging size");
constexpr int KP = (PW::NS + 2 * NT - 1) / (2 * NT);  // staged pairs per thread (9)
static_assert(2 * NT * (KP - 1) + 2 * NT - 1 >= PW::NS - 1, "staging coverage");


// Prefetch of one tile's inputs: branch-free 16-B loads at clamped addresses, so
// the loads stay in flight (a branchy prefetch makes the compiler merge register
// copies behind an s_waitcnt vmcnt(0)). Tiles that reach before x[0] or past
// x[n-1] are re-loaded exactly (history / zero padding) at staging time.
// ---- front, wave-independent form ----------------------------------------------
// One wave per workgroup and no s_barrier anywhere: every LDS hand-off is inside
// one wave (DS operations of a wave complete in order; wave_lds_fence keeps the
// compiler from reordering around them). Each wave owns a contiguous range of
// decimated outputs [A, B) and walks it in tiles of TW = 64R outputs, one tile's
// 8 TW new inputs prefetched into registers while the previous tile computes.
// Consecutive tiles share 17 polyphase rows (the FIR's Q-row history): they are
// copied inside LDS from the tail to the head of each row, times e^{-j theta NEW}
// so that every tile is NCO-mixed relative to its own origin (the tile's common
// phasor multiplies its outputs, as in the persistent form).
// R = 6: lanes read 6-output windows at a 48-B stride (three 16-B bank slots, odd,
// so the 16-lane ds_read_b128 groups are conflict-free); 11 b128 reads and 96
// packed FMAs per lane and phase; 25.7 KB of LDS per wave (6 waves per CU).
template <int R>
struct Fw {
  static constexpr int TW = 64 * R;      // decimated outputs per tile
  static constexpr int NEW = M * TW;     // inputs entering per tile
  static constexpr int KL = NEW / 128;   // 2-sample loads per lane per tile (4R)
  static constexpr int LR = TW + Q + 2;  // row pitch: rows hold i = 0 .. TW+Q (+1 pad)
  static constexpr int WIN = (R + Q) / 2;  // b128 window reads per lane and phase
  static constexpr int LDS_F2 = M * LR;
  static_assert(LR % 16 == 2, "row pitch = 2 mod 16 (phase-scattered b64 stores)");
  static_assert((R % 2) == 0 && NEW <= kWbfmNS, "phasor table covers the tile");
};


// Lane l receives lane l-1's value; lane 0 receives `first` (DPP wave_shr:1).
__device__ __forceinline__ float wave_shr1(float v, float first) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(first), __float_as_int(v), 0x138,
                                                    0xf, 0xf, false));
}

// Prefetch of a tile's new samples x[B + o], o = 2l + 128k, B = porg + 8Q.
// Large inputs (CLAMP = false, n >= 2 NEW): the uniform base is clamped into
// [0, n - NEW], so interior tiles load exactly and one offset register serves
// every load; a boundary tile then loads shifted samples, all of which the
// staging fixup rewrites. Small inputs (CLAMP = true): per-lane clamp of the
// 32-bit offset to [0, n-2] (only the out-of-range samples are wrong).
template <int R, bool A16, bool CLAMP>
__device__ __forceinline__ void front2_load(const f2* __restrict__ x, long long n, long long porg,
                                            int l, f2 (&v)[Fw<R>::KL][2]) {
  const long long B = porg + 8 * Q;
  const f2* __restrict__ xb;
  int lo = 0, hi = 0;
  if constexpr (CLAMP) {
    constexpr long long kSat = 1LL << 30;
    lo = static_cast<int>(max(-B, -kSat));                                   // even
    hi = static_cast<int>(min(max((n - 2 - B) & ~1LL, -kSat), kSat));        // even, >= lo
    xb = x + B;
  } else {
    xb = x + min(max(B, 0LL), (n - Fw<R>::NEW) & ~1LL);
  }
#pragma unroll
  for (int k = 0; k < Fw<R>::KL; ++k) {
    const int o = CLAMP ? min(max(2 * l + 128 * k, lo), hi) : 2 * l + 128 * k;
    if constexpr (A16) {
      // Nontemporal: the input is read once; streaming it past the caches keeps
      // the phi / output lines resident (measured 6.9 vs 6.0 TB/s, membench).
      const f4 w = __builtin_nontemporal_load(reinterpret_cast<const f4*>(xb + o));
      v[k][0] = f2{w.x, w.y};
      v[k][1] = f2{w.z, w.w};
    } else {
      v[k][0] = xb[o];
      v[k][1] = xb[o + 1];
    }
  }
}

// One polyphase phase: window w (b128 pairs of U[c][R l ..]) against taps t.
template <int R>
__device__ __forceinline__ void front2_phase(const f4 (&w)[Fw<R>::WIN], const float (&t)[Q], f2 (&d)[R]) {
#pragma unroll
  for (int h = 0; h < Fw<R>::WIN; ++h) {
    const f2 w0 = f2{w[h].x, w[h].y}, w1 = f2{w[h].z, w[h].w};
    // window entry m -> output rho uses tap q = rho + Q - m
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int q0 = r + Q - 2 * h, q1 = r + Q - 2 * h - 1;
      if (q0 >= 0 && q0 < Q) d[r] = fma2(splat2(t[q0]), w0, d[r]);
      if (q1 >= 0 && q1 < Q) d[r] = fma2(splat2(t[q1]), w1, d[r]);
    }
  }
}

template <int R>
__device__ __forceinline__ void front2_window(const f2* __restrict__ U, int l, int c, f4 (&w)[Fw<R>::WIN]) {
  const f4* row = reinterpret_cast<const f4*>(U + c * Fw<R>::LR + R * l);
#pragma unroll
  for (int h = 0; h < Fw<R>::WIN; ++h) w[h] = row[h];
}
__device__ __forceinline__ void front2_taps(const float* __restrict__ g, int c, float (&t)[Q]) {
#pragma unroll
  for (int q = 0; q < Q; ++q) t[q] = g[c * Q + q];
}

// Polyphase FIR over the 8 phases (rolled: SGPR taps stay at 16 per phase).
template <int R>
__device__ __forceinline__ void front2_decim(const f2* __restrict__ U, int l, const float* __restrict__ g,
                                             f2 (&d)[R]) {
#pragma unroll
  for (int r = 0; r < R; ++r) d[r] = f2{0.0f, 0.0f};
#pragma unroll 1
  for (int c = 0; c < M; ++c) {
    f4 w[Fw<R>::WIN];
    float t[Q];
    front2_window<R>(U, l, c, w);
    front2_taps(g, c, t);
    front2_phase<R>(w, t, d);
  }
}

#ifndef ORION_SEG2_PF1
#define ORION_SEG2_PF1 0  // 1: k_wbfm_seg2 keeps one tile of inputs in flight, not two
#endif
#ifndef ORION_SEG2_PHGEN
#define ORION_SEG2_PHGEN 0  // 1: k_wbfm_seg2 forms staging phasors per tile (32 fewer VGPRs)
#endif
template <int R, bool A16, int ABL, bool CLAMP = false>
__global__ __launch_bounds__(64, R <= 2 ? 3 : 2) void k_wbfm_front2(const WbfmArgs a, const WbfmFrontConst C,
                                                    long long L, int wpc) {
  using G = Fw<R>;
  __shared__ __attribute__((aligned(16))) f2 U[G::LDS_F2];
  const int l = threadIdx.x;
  const int ch = blockIdx.x / wpc;
  const long long A = static_cast<long long>(blockIdx.x - ch * wpc) * L;
  const long long B = min(A + L, a.n_dec);
  if (A >= B) return;
  const int ntiles = static_cast<int>((B - A + G::TW) / G::TW);  // outputs A-1 .. B-1

  const f2* __restrict__ tabc = a.tab + static_cast<long long>(ch) * kWbfmNS;
  const bool tiny = a.n < 2;
  const f2* __restrict__ xc = a.x + ch * a.x_stride;
  const f2* __restrict__ xl = tiny ? a.hist_in + ch * kWbfmHist : xc;  // clamp target
  const long long nl = tiny ? kWbfmHist : a.n;
  const f2* __restrict__ hc = a.hist_in + ch * kWbfmHist;
  const uint64_t step = a.step[ch];
  const float* __restrict__ ci = a.carry_in + ch * kWbfmCarry;
  const f2 cprev = f2{ci[4], ci[5]};
  float* __restrict__ phi = a.phi + ch * a.phi_stride;

  // Lane phasors: new samples p = 8Q + 2l + 128k (k < KL) -> e^{j theta p} =
  // tb * tab[128k]; halo samples p = 2l, 2l+1 of the first tile -> tab[p].
  const f4 tv = *reinterpret_cast<const f4*>(tabc + 8 * Q + 2 * l);
  const f2 tb0 = f2{tv.x, tv.y}, tb1 = f2{tv.z, tv.w};
  // Lane phasors e^{j theta p} of the new samples, p = 8Q + 2l + 128k (+1):
  // the same for every tile (each tile is mixed relative to its own origin).
  f2 ph[R <= 2 ? G::KL : 1][2];
  if constexpr (R <= 2) {
#pragma unroll
    for (int k = 0; k < G::KL; ++k) {
      const f2 ek = tabc[128 * k];
      ph[k][0] = cmul(tb0, ek);
      ph[k][1] = cmul(tb1, ek);
    }
  }
  const f2 cn = tabc[G::NEW];
  const f2 corr = f2{cn.x, -cn.y};  // e^{-j theta NEW}
  const int c0 = (-2 * l) & 7, c1 = (-2 * l - 1) & 7;
  const int s0 = c0 * G::LR + (8 * Q + 2 * l + c0) / 8;
  const int s1 = c1 * G::LR + (8 * Q + 2 * l + 1 + c1) / 8;

  long long porg = 8LL * (A - 1 - Q);  // x index of staged sample p = 0
  f2 v[G::KL][2];
  if constexpr (ABL & 1) {
#pragma unroll
    for (int k = 0; k < G::KL; ++k) v[k][0] = v[k][1] = f2{static_cast<float>(l), 1.0f};
  } else {
    front2_load<R, A16, CLAMP>(xl, nl, porg, l, v);
  }
  {  // halo rows of the first tile (p = 2l, 2l+1), mixed with tab[p]
    const f4 th = *reinterpret_cast<const f4*>(tabc + 2 * l);
    const f2 x0 = load_hist(xc, a.n, hc, kWbfmHist, porg + 2 * l);
    const f2 x1 = load_hist(xc, a.n, hc, kWbfmHist, porg + 2 * l + 1);
    U[c0 * G::LR + (2 * l + c0) / 8] = cmul_rot(x0, f2{th.x, th.y});
    U[c1 * G::LR + (2 * l + 1 + c1) / 8] = cmul_rot(x1, f2{th.z, th.w});
  }

  f2 Sv = f2{1.0f, 0.0f};  // lane m: common phasor of tile nb + m
  int nb = 0;
  f2 carry = f2{0.0f, 0.0f};
  for (int n = 0; n < ntiles; ++n, porg += G::NEW) {
    const long long jd0 = A - 1 + static_cast<long long>(n) * G::TW;
    if (n == nb) {  // tile phasors for the next 64 tiles, one per lane
      Sv = phasor_q64(static_cast<uint64_t>(a.k0 + porg + 1 + static_cast<long long>(l) * G::NEW), step);
      nb += 64;
    }
    // ---- halo: the previous tile's last 17 rows -> rows 0..16 (x e^{-j theta NEW}) ----
    if (n > 0 && !(ABL & 256)) {
#pragma unroll
      for (int r2 = 0; r2 < 2; ++r2) {
        const int e = l + 64 * r2;
        if (e < 72) {
          const int c = e / 9, h = e - 9 * c;
          const f4 w = *reinterpret_cast<const f4*>(U + c * G::LR + G::TW + 2 * h);
          const f2 y0 = cmul(f2{w.x, w.y}, corr), y1 = cmul(f2{w.z, w.w}, corr);
          *reinterpret_cast<f4*>(U + c * G::LR + 2 * h) = f4{y0.x, y0.y, y1.x, y1.y};
        }
      }
      wave_lds_fence();
    }
    // ---- stage the new samples: NCO mix, polyphase scatter ----
    const bool bnd = porg < 0 || porg + 8LL * (G::TW + Q) > a.n;
    if constexpr (R <= 2) {  // lane phasors precomputed once per wave (2 KL registers pairs)
#pragma unroll
      for (int k = 0; k < G::KL; ++k) {
        if constexpr (ABL & 4) {
          U[s0 + 16 * k] = v[k][0];
          U[s1 + 16 * k] = v[k][1];
        } else {
          U[s0 + 16 * k] = cmul_rot_pk(v[k][0], ph[k][0]);
          U[s1 + 16 * k] = cmul_rot_pk(v[k][1], ph[k][1]);
          if (k % 4 == 3) asm volatile("" ::: "memory");  // bound the live temporaries
        }
      }
    } else {
      // Opaque per tile: stops the compiler from hoisting all 2*KL lane phasors
      // tb * tab[128k] out of the tile loop (96 live VGPRs for R = 6).
      int opaque_zero;
      asm volatile("s_mov_b32 %0, 0" : "=s"(opaque_zero));
      const f2* tabk = tabc + opaque_zero;
#pragma unroll
      for (int k = 0; k < G::KL; ++k) {
        const f2 x0 = v[k][0], x1 = v[k][1];
        if constexpr (ABL & 4) {
          U[s0 + 16 * k] = x0;
          U[s1 + 16 * k] = x1;
        } else {
          const f2 ek = tabk[128 * k];
          U[s0 + 16 * k] = cmul_rot_pk(x0, cmul(tb0, ek));
          U[s1 + 16 * k] = cmul_rot_pk(x1, cmul(tb1, ek));
        }
      }
    }
    // ---- prefetch the next tile (lands during this tile's FIR) ----
    // The compiler fence keeps the new loads below the staging stores, so the
    // current and the next tile's registers are never live together.
    asm volatile("" ::: "memory");
    if constexpr (!(ABL & 1))
      if (n + 1 < ntiles) front2_load<R, A16, CLAMP>(xl, nl, porg + G::NEW, l, v);
    if (bnd) {
      // Tile reaching before x[0] or past x[n-1]: the clamped prefetch staged
      // wrong samples there; rewrite exactly those slots (history / zeros).
      wave_lds_fence();
#pragma unroll 1
      for (int p = 8 * Q + l; p < 8 * (G::TW + Q); p += 64) {
        const long long P = porg + p;
        if (!CLAMP || P < 0 || P >= a.n) {  // unclamped loads may be shifted: rewrite all
          const int c = (-p) & 7;
          U[c * G::LR + (p + c) / 8] = cmul_rot(load_hist(xc, a.n, hc, kWbfmHist, P), tabc[p]);
        }
      }
    }
    wave_lds_fence();

    // ---- polyphase FIR: outputs jd0 + R l + rho ----
    f2 d[R];
    if constexpr (ABL & 2) {
#pragma unroll
      for (int r = 0; r < R; ++r) d[r] = U[R * l + r];
    } else {
      front2_decim<R>(U, l, C.g, d);
    }
    if constexpr (!(ABL & 1024)) {
      const int sl = n - (nb - 64);
      const f2 S = f2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(Sv.x), sl)),
                      __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Sv.y), sl))};
#pragma unroll
      for (int r = 0; r < R; ++r) d[r] = cmul(d[r], S);
    }
    if (n == 0 && A == 0 && l == 0) d[0] = cprev;  // d[-1]: carried from the previous call

    // ---- FM discriminator (fm.rs:60-68) ----
    const f2 pv = (ABL & 1024) ? d[0] : f2{wave_shr1(d[R - 1].x, carry.x), wave_shr1(d[R - 1].y, carry.y)};
    // Emitted outputs: tile-relative index e = R l + r in [elo, ehi) (32-bit).
    const int elo = static_cast<int>(max(A - jd0, 0LL));
    const int ehi = static_cast<int>(min(B - jd0, static_cast<long long>(G::TW)));
    float* __restrict__ phit = phi + jd0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int e = R * l + r;
      const f2 pr = r == 0 ? pv : d[r - 1];
      if constexpr (ABL & 128) {  // timing only: coalesced lane order, wrong data
        const int ec = l + 64 * r;
        if (ec >= elo && ec < ehi) phit[ec] = (ABL & 8) ? d[r].x + pr.y : fm_disc_pk(d[r], pr, C.k);
      } else if constexpr (ABL & 512) {  // timing only: no stores (kept alive)
        const float o = (ABL & 8) ? d[r].x + pr.y : fm_disc_pk(d[r], pr, C.k);
        if (o == 1234.5f) phit[e] = o;
      } else if (e >= elo && e < ehi) {
        if constexpr (ABL & 8) phit[e] = d[r].x + pr.y;
        else phit[e] = fm_disc_pk(d[r], pr, C.k);
      }
    }
    carry = f2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(d[R - 1].x), 63)),
               __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d[R - 1].y), 63))};
    // ---- carried state: last decimated sample and raw history ----
    if (jd0 <= a.n_dec - 1 && a.n_dec - 1 < jd0 + G::TW) {
      const int rl = static_cast<int>(a.n_dec - 1 - jd0);
      float* co = a.carry_out + ch * kWbfmCarry;
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (R * l + r == rl) {
          co[4] = d[r].x;
          co[5] = d[r].y;
          co[6] = 0.0f;
          co[7] = 0.0f;
        }
#pragma unroll
      for (int t2 = 0; t2 < kWbfmHist / 64; ++t2) {
        const int t = l + 64 * t2;
        a.hist_out[ch * kWbfmHist + t] = load_hist(xc, a.n, hc, kWbfmHist, a.n - kWbfmHist + t);
      }
    }
  }
}

// ---- back kernel ------------------------------------------------------------
// One workgroup (256 lanes) per block of kBackA = 4096 audio outputs [a0, a0+4096),
// split into two halves 2048 apart. Each half runs LpCascade over its 2048 phi
// plus kBackW = 510 samples of zero-state warm-up (double pole, r = 0.953: the
// transient is < 2e-8 of the state after 510 samples); lane l owns chunk l
// (kBackC = 10 samples) of both halves and runs them as one packed float2
// recurrence (v_pk_* ops: the reference's f32 TDF-II roundings, two chunks at
// once). Chunk states come from an f64 Kogge-Stone scan per half.
// Local index j = i - a0. Half A covers j in [-510, 2050), half B j + 2048.
// Block 0 has no warm-up data: its half-A lanes 0..50 see zero input and lane
// 50's aggregate is replaced by the IIR state carried from the previous call,
// which then enters lane 51 (j = 0) exactly.
// LDS: F (phi, j in [-510, 4098), zero outside [0, n_dec)) for pass 1, aliased
// by P[j] = (f[j], f[j + 2048]) for j in [-124, 2048), the audio FIR's pair image
// (one v_pk_fma_f32 applies a tap to both halves), one pad slot per 8 pairs
// (lane stride 9 pairs = 18 dwords: conflict-free ds_read_b64).
constexpr int kHalf = kBackA / 2;
constexpr int kFSpan = kBackSpan + kHalf;                 // 4608 staged phi
constexpr int kPairs = kHalf + 124;                       // j in [-124, 2048)
__host__ __device__ constexpr int ppos(int e) { return e + (e >> 3); }  // e = j + 124
constexpr int kPDummy = ppos(kPairs) + 1;                 // sink for unneeded warm-up pairs
constexpr int kPSlots = kPDummy + 1;
constexpr int kBackLdsBytes = (kPSlots * 8 > kFSpan * 4 ? kPSlots * 8 : kFSpan * 4);
static_assert(kBackW % kBackC == 0 && 2 * kBackSpan >= kBackA + 2 * kBackW, "back geometry");

// BiquadK::step on two independent streams: identical roundings, packed ops.
struct Biquad2 {
  f2 b0, b1, b2, a1, a2;
  __device__ __forceinline__ f2 step(f2& z1, f2& z2, f2 x) const {
    const f2 y = __builtin_elementwise_fma(x, b0, z1);
    z1 = __builtin_elementwise_fma(x, b1, z2) - a1 * y;
    z2 = x * b2 - a2 * y;
    return y;
  }
  __device__ __forceinline__ f2 lp4(f2 (&s)[4], f2 x) const {
    const f2 y0 = step(s[0], s[1], x);
    return step(s[2], s[3], y0);
  }
};

template <int ABL>
__global__ __launch_bounds__(NT, 4) void k_wbfm_back(const WbfmArgs a, const WbfmBackConst C) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[kBackLdsBytes];
  __shared__ double tot[4][2][4];
  float* F = reinterpret_cast<float*>(lds);
  f2* P = reinterpret_cast<f2*>(lds);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int ch = blockIdx.y;
  const long long a0 = static_cast<long long>(blockIdx.x) * kBackA;
  const long long a_end = min(a0 + kBackA, a.n_dec);
  const bool first = blockIdx.x == 0;
  const bool last = a_end == a.n_dec;
  const float* __restrict__ phi = a.phi + ch * a.phi_stride;
  const float* __restrict__ ci = a.carry_in + ch * kWbfmCarry;
  const Biquad2 bq{splat2(C.b0), splat2(C.b1), splat2(C.b2), splat2(C.a1), splat2(C.a2)};

  // ---- stage phi (zero outside [0, n_dec)) ----
  for (int e = t; e < kFSpan; e += NT) {
    const long long i = a0 - kBackW + e;
    F[e] = (i >= 0 && i < a.n_dec) ? phi[i] : 0.0f;
  }
  __syncthreads();
  f2 xs[kBackC];  // (half A, half B) inputs of this lane's chunks
#pragma unroll
  for (int i = 0; i < kBackC; i += 2) {  // b64 pairs, 40-B lane stride: conflict-free
    const f2 u = *reinterpret_cast<const f2*>(F + kBackC * t + i);
    const f2 w = *reinterpret_cast<const f2*>(F + kBackC * t + i + kHalf);
    xs[i] = f2{u.x, w.x};
    xs[i + 1] = f2{u.y, w.y};
  }

  // ---- pass 1: zero-state chunk aggregates, f64 scan per half ----
  f2 s[4] = {f2{0, 0}, f2{0, 0}, f2{0, 0}, f2{0, 0}};
  if constexpr (!(ABL & 32)) {
#pragma unroll
    for (int i = 0; i < kBackC; ++i) (void)bq.lp4(s, xs[i]);
  }
  double q[2][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    q[0][k] = s[k].x;
    q[1][k] = s[k].y;
  }
  if (first && t == kBackW / kBackC - 1)  // state at j = 0 (previous call) enters lane 51
#pragma unroll
    for (int k = 0; k < 4; ++k) q[0][k] = ci[k];
  if constexpr (!(ABL & 32)) {
#pragma unroll 1
    for (int st = 0; st < 6; ++st) {
      const int d = 1 << st;
      double o[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int k = 0; k < 4; ++k) o[h][k] = __shfl_up(q[h][k], d, 64);
      if (lane >= d) {
        matvec_acc<4>(C.pw + st * 16, o[0], q[0]);
        matvec_acc<4>(C.pw + st * 16, o[1], q[1]);
      }
    }
  }
  if (lane == 63)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < 4; ++k) tot[wave][h][k] = q[h][k];
  __syncthreads();  // also: every lane holds its inputs (F is dead, P may overwrite it)

  // entering state of this lane's chunks: lanemats[lane] * (state entering the
  // wave) + the exclusive in-wave prefix
  f2 ef[4];
  {
    double cw[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    for (int w = 0; w < wave; ++w) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        double vv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) vv[k] = tot[w][h][k];
        matvec_acc<4>(C.mw, cw[h], vv);
#pragma unroll
        for (int k = 0; k < 4; ++k) cw[h][k] = vv[k];
      }
    }
    double e[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double o = __shfl_up(q[h][k], 1, 64);
        e[h][k] = lane == 0 ? 0.0 : o;
      }
    matvec_acc<4>(a.lanemats + lane * 16, cw[0], e[0]);
    matvec_acc<4>(a.lanemats + lane * 16, cw[1], e[1]);
#pragma unroll
    for (int k = 0; k < 4; ++k) ef[k] = f2{static_cast<float>(e[0][k]), static_cast<float>(e[1][k])};
  }
  if constexpr (ABL & 32) {
#pragma unroll
    for (int k = 0; k < 4; ++k) ef[k] = f2{0, 0};
  }

  // ---- pass 2: the reference's f32 recurrence from the entering state ----
  // Pairs j < -124 (warm-up not needed by the FIR) and, in block 0, j < 0 (the
  // previous call's f values are written below) go to a dummy slot.
  const int jlo = first ? 0 : -124;
  const int j0 = kBackC * t - kBackW;
  if (!last) {
#pragma unroll
    for (int i = 0; i < kBackC; ++i) {
      const int j = j0 + i;
      const f2 f = (ABL & 32) ? xs[i] * ef[0] : bq.lp4(ef, xs[i]);
      P[j >= jlo ? ppos(j + 124) : kPDummy] = f;
    }
  } else {
    // last block: also capture the IIR state after sample n_dec - 1
    const int jl = static_cast<int>(a.n_dec - 1 - a0);  // local index of the last sample
    float cap[4] = {0, 0, 0, 0};
    bool have = false;
#pragma unroll
    for (int i = 0; i < kBackC; ++i) {
      const int j = j0 + i;
      const f2 f = (ABL & 32) ? xs[i] * ef[0] : bq.lp4(ef, xs[i]);
      P[j >= jlo ? ppos(j + 124) : kPDummy] = f;
      if (j == jl && jl < kHalf) {  // half A owns j < 2048 (its tail past 2048 is B's)
#pragma unroll
        for (int k = 0; k < 4; ++k) cap[k] = ef[k].x;
        have = true;
      }
      if (j + kHalf == jl && j >= 0) {  // half B owns j >= 2048 (its warm-up is A's)
#pragma unroll
        for (int k = 0; k < 4; ++k) cap[k] = ef[k].y;
        have = true;
      }
    }
    if (have) {
      float* co = a.carry_out + ch * kWbfmCarry;
#pragma unroll
      for (int k = 0; k < 4; ++k) co[k] = cap[k];
    }
  }
  // Pairs j in [-124, 0): .y = f[j + 2048] came from half B's warm-up; the exact
  // value is half A's (converged) f at 1924 .. 2047. Block 0: .x = f[-124 .. -1]
  // of the previous call.
  __syncthreads();
  if (t < 124) {
    P[ppos(t)].y = P[ppos(t + kHalf)].x;
    if (first) P[ppos(t)].x = ci[8 + 4 + t];
  }
  __syncthreads();

  // ---- audio FIR (fir.rs:57-66, quirk-mapped taps) ----
  // Lane t owns outputs j = 8t + i and j + 2048 (i < 8) as float2 pairs. Output
  // j, tap k = 16 kb + kk reads f[j - k]: window index m = i + 15 - kk of the
  // 23 pairs starting at e = 8t - 16kb - 15 + 124 = 8(t - 2kb) + 109; with
  // ppos, slot = 9(t - 2kb) + 109 + m + ((109 + m) >> 3): a per-lane base plus
  // compile-time offsets.
  {
    constexpr int R = 8, KA = 128;
    f2 acc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = f2{0.0f, 0.0f};
    if constexpr (ABL & 16) {
#pragma unroll
      for (int i = 0; i < R; ++i) acc[i] = P[ppos(8 * t + i + 124)];
    } else {
#pragma unroll 1
      for (int kb = 0; kb < KA / 16; ++kb) {
        const f2* __restrict__ Pl = P + 9 * (t - 2 * kb) + 109;
        f2 w[R + 15];
#pragma unroll
        for (int m = 0; m < R + 15; ++m) w[m] = Pl[m + ((109 + m) >> 3)];
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
          const f2 tap = splat2(C.a[16 * kb + kk]);
#pragma unroll
          for (int i = 0; i < R; ++i) acc[i] = fma2(tap, w[i + 15 - kk], acc[i]);
        }
      }
    }
    float* __restrict__ y = a.y + ch * a.y_stride + a0;
    const int nv = static_cast<int>(a_end - a0);
    if (nv == kBackA) {
      float4* ya = reinterpret_cast<float4*>(y + R * t);
      float4* yb = reinterpret_cast<float4*>(y + kHalf + R * t);
      if ((reinterpret_cast<uintptr_t>(y) & 15) == 0) {
        ya[0] = float4{acc[0].x, acc[1].x, acc[2].x, acc[3].x};
        ya[1] = float4{acc[4].x, acc[5].x, acc[6].x, acc[7].x};
        yb[0] = float4{acc[0].y, acc[1].y, acc[2].y, acc[3].y};
        yb[1] = float4{acc[4].y, acc[5].y, acc[6].y, acc[7].y};
      } else {
#pragma unroll
        for (int i = 0; i < R; ++i) {
          y[R * t + i] = acc[i].x;
          y[kHalf + R * t + i] = acc[i].y;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int j = R * t + i;
        if (j < nv) y[j] = acc[i].x;
        if (j + kHalf < nv) y[j + kHalf] = acc[i].y;
      }
    }
  }
  if (last && t < 128) {  // last 128 f values (fhist of the next call)
    const int j = static_cast<int>(a.n_dec - 128 + t - a0);
    float f;
    if (j >= 0) f = j < kHalf ? P[ppos(j + 124)].x : P[ppos(j - kHalf + 124)].y;
    else f = j >= -124 ? P[ppos(j + 124)].x : ci[8 + 128 + j];  // reaches into the carried history
    a.carry_out[ch * kWbfmCarry + 8 + t] = f;
  }
}

// ---- fused chain -------------------------------------------------------------
// k_wbfm_fused<N>: the whole chain in one kernel, no phi round trip through HBM.
// One wave per range of L = 128 N decimated outputs [A, A+L) of a channel
// (waves of one channel are consecutive blockIdx). Per wave:
//   1. front (as k_wbfm_front2, tiles aligned at A; input prefetched two tiles
//      ahead): N tiles -> phi in LDS. phi[A] needs d[A-1], the previous range's
//      last decimated sample;
//   2. hand-off 1: publish d[A+L-1], wait for the predecessor's, finish phi[A];
//   3. LpCascade zero-state pass over the range (two halves of L/2 as one packed
//      float2 recurrence, f64 Kogge-Stone per half) -> the range's zero-state
//      aggregate a_w;
//   4. hand-off 2: publish a_w, wait for a_{w-1}. The state entering the range
//      is sum_k A^{L(k-1)} a_{w-k} = a_{w-1}: the host only selects this kernel
//      when ||A^L|| is negligible (f32 cannot see the remainder);
//   5. the reference's f32 recurrence from the entering states -> the audio
//      FIR's pair image P[j] = (f[j], f[j+L/2]) (as in k_wbfm_back);
//   6. hand-off 3: publish f[A+L-128 .. A+L), wait for the predecessor's last
//      128 -> the FIR history; 7. audio FIR -> y.
// Each hand-off publishes before it waits and only needs the predecessor's
// previous stage, so no wait chain is longer than three ranges; waves are
// dispatched in blockIdx order per XCD, so the predecessor is resident or done.
// Waits are bounded (the kernel never hangs; a timeout sets *err). Hand-off data
// use agent-scope relaxed atomics (coherent across the XCDs' L2s), ordered by an
// s_waitcnt vmcnt(0) before the flag store.
namespace fu {
using G = Fw<2>;
// debug timing: lane 0 records s_memrealtime (100 MHz) at phase boundaries
__device__ __forceinline__ void trace(const WbfmArgs& a, int r, int point) {
  if (a.trace && (threadIdx.x & 63) == 0)
    a.trace[static_cast<long long>(r) * kFuTracePoints + point] =
        static_cast<long long>(__builtin_amdgcn_s_memrealtime());
}
constexpr int PB = kFuTail;  // FIR history pairs (j >= -128)

template <int N>
struct Geo {
  static constexpr int L = 128 * N;           // outputs per range
  static constexpr int NH = L / 2;            // per IIR half
  static constexpr int CH = NH / 64;          // IIR chunk per lane per half = FIR outputs per lane per half
  static_assert((CH & (CH - 1)) == 0 && CH >= 8, "chunk a power of two");
  // FIR pair slots: one pad per CH pairs -> lane stride CH+1 pairs (2(CH+1) dwords:
  // 2 x odd, so the ds_read_b64 of 32 lanes hit distinct bank pairs)
  __host__ __device__ static constexpr int pslot(int e) { return e + e / CH; }
  static constexpr int PSlots = pslot(NH + PB) + 1;
  static constexpr int UPhiBytes = G::LDS_F2 * 8 + L * 4;   // front image + phi
  static constexpr int LdsBytes = (PSlots * 8 > UPhiBytes ? PSlots * 8 : UPhiBytes);
  static constexpr int WavesPerSimd = N <= 8 ? 3 : 2;
};

__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// This wave's stores have completed (reached the agent coherence point).
__device__ __forceinline__ void stores_done() { __builtin_amdgcn_s_waitcnt(0x0F70); }
__device__ __forceinline__ void publish(uint32_t* flag, uint32_t epoch, int l) {
  stores_done();
  if (l == 0) st_agent(flag, epoch);
}
__device__ __forceinline__ void wait_for(const uint32_t* flag, uint32_t epoch, int* err) {
  for (int it = 0; it < (1 << 21); ++it) {
    if (ld_agent(flag) == epoch) {
      asm volatile("" ::: "memory");
      return;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double u2d(uint32_t lo, uint32_t hi) {
  return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}
}  // namespace fu

// One front tile (tiles aligned at the range start). The registers v hold this
// tile's prefetched inputs on entry; on exit they hold the loads issued for the
// tile two ahead (pf), possibly in the next range, possibly another channel.
struct FuTile {
  const WbfmArgs& a;
  const WbfmFrontConst& C;
  f2* U;
  float* Phi;
  const float* Gt;  // decimator taps in LDS (phase-major)
  const f2* xc;
  const f2* hc;
  const f2* tabc;
  int ch, l, s0, s1;
  f2 corr;
  bool first;  // the channel's first range: d[A-1] is the carried sample
};
struct FuPrefetch {  // where the tile two ahead starts
  const f2* xl;
  long long nl, porg;
  bool on;
};

#ifndef ORION_FU_ABL
#define ORION_FU_ABL 0  // timing experiments only (separate builds): 2 no decim FIR, 4 no staging
#endif

// Per-lane staging phasors of a tile, ph(k, r) = e^{j theta (8Q + 2l + r + 128 k)}:
// held in 32 registers (PhArr) or formed per tile from the lane's two base
// phasors and the uniform e^{j theta 128 k} (PhGen: same products, same bits).
struct PhArr {
  const f2 (&p)[8][2];
  __device__ __forceinline__ f2 operator()(int k, int r) const { return p[k][r]; }
};
struct PhGen {
  f2 tb0, tb1;
  const f2* __restrict__ tabc;
  __device__ __forceinline__ f2 operator()(int k, int r) const { return cmul(r ? tb1 : tb0, tabc[128 * k]); }
  // a copy the compiler cannot see through: keeps the products inside the tile
  // loop (hoisted, they would occupy the 32 registers this form saves)
  __device__ __forceinline__ PhGen opaque() const {
    PhGen q = *this;
    asm volatile("" : "+v"(q.tb0.x), "+v"(q.tb0.y), "+v"(q.tb1.x), "+v"(q.tb1.y));
    return q;
  }
};

template <bool A16, bool CLAMP, class PH>
__device__ __forceinline__ void fu_tile(const FuTile& T, int n, long long porg, long long jd0, const PH& ph,
                                        f2 (&v)[8][2], const FuPrefetch& pf, f2 Sv, f2& carry, f2& dA,
                                        float* __restrict__ phit, int svi, bool copy_halo = true) {
  using G = fu::G;
  constexpr int R = 2;
  f2* __restrict__ U = T.U;
  const int l = T.l;
  if (n > 0 && copy_halo) {
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      const int e = l + 64 * r2;
      if (e < 72) {
        const int c = e / 9, h = e - 9 * c;
        const f4 w = *reinterpret_cast<const f4*>(U + c * G::LR + G::TW + 2 * h);
        const f2 y0 = cmul(f2{w.x, w.y}, T.corr), y1 = cmul(f2{w.z, w.w}, T.corr);
        *reinterpret_cast<f4*>(U + c * G::LR + 2 * h) = f4{y0.x, y0.y, y1.x, y1.y};
      }
    }
    wave_lds_fence();
  }
  const bool bnd = porg < 0 || porg + 8LL * (G::TW + Q) > T.a.n;
#pragma unroll
  for (int k = 0; k < G::KL; ++k) {
    if constexpr (ORION_FU_ABL & 4) {  // timing experiment: no staging (loads kept alive)
      if (k == 0) U[T.s0] = v[0][0] + v[1][0] + v[2][0] + v[3][0] + v[4][0] + v[5][0] + v[6][0] + v[7][0];
      if (k == 0) U[T.s1] = v[0][1] + v[1][1] + v[2][1] + v[3][1] + v[4][1] + v[5][1] + v[6][1] + v[7][1];
      continue;
    }
    U[T.s0 + 16 * k] = cmul_rot_pk(v[k][0], ph(k, 0));
    U[T.s1 + 16 * k] = cmul_rot_pk(v[k][1], ph(k, 1));
    if (k % 4 == 3) asm volatile("" ::: "memory");
  }
  asm volatile("" ::: "memory");
  // unconditional: a conditional prefetch makes the compiler's wait counting
  // assume the other buffer's loads may be absent and drain them (vmcnt(0))
  front2_load<R, A16, CLAMP>(pf.xl, pf.nl, pf.porg, l, v);
  if (bnd) {
    // Tile reaching before x[0] or past x[n-1]: rewrite the new samples (and, in
    // a range's first tile, the halo rows) exactly from the history / zeros.
    wave_lds_fence();
#pragma unroll 1
    for (int p = (n == 0 ? 0 : 8 * Q) + l; p < 8 * (G::TW + Q); p += 64) {
      const long long Pp = porg + p;
      if (!CLAMP || Pp < 0 || Pp >= T.a.n || p < 8 * Q) {
        const int c = (-p) & 7;
        U[c * G::LR + (p + c) / 8] = cmul_rot(load_hist(T.xc, T.a.n, T.hc, kWbfmHist, Pp), T.tabc[p]);
      }
    }
  }
  wave_lds_fence();
  f2 d[R];
  if constexpr (ORION_FU_ABL & 2) {  // timing experiment: no decimating FIR
    d[0] = U[l];
    d[1] = U[l + 64];
  } else {
    front2_decim<R>(U, l, T.C.g, d);
  }
  const f2 S = f2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(Sv.x), svi)),
                  __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Sv.y), svi))};
#pragma unroll
  for (int r = 0; r < R; ++r) d[r] = cmul(d[r], S);
  if (n == 0 && !T.first) {
    // d[A-1], the previous range's last output, from this tile's image (rows
    // i = 0..15; the range setup staged U[c][0], c >= 1): taps 2l, 2l+1 per
    // lane, summed over the wave.
    f2 acc = f2{0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int k = 2 * l + t, c = k & 7, q = k >> 3;
      acc = fma2(splat2(T.Gt[c * Q + q]), U[c * G::LR + 15 - q], acc);  // LDS taps: no vmcnt drain
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
      acc += f2{__shfl_xor(acc.x, off, 64), __shfl_xor(acc.y, off, 64)};
    carry = cmul(acc, S);
  }
  const f2 pv = f2{wave_shr1(d[R - 1].x, carry.x), wave_shr1(d[R - 1].y, carry.y)};
  phit[2 * l] = fm_disc_pk_rcp(d[0], pv, T.C.k);
  phit[2 * l + 1] = fm_disc_pk_rcp(d[1], d[0], T.C.k);
  if (n == 0) dA = d[0];
  carry = f2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(d[R - 1].x), 63)),
             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d[R - 1].y), 63))};
  const WbfmArgs& a = T.a;
  if (jd0 <= a.n_dec - 1 && a.n_dec - 1 < jd0 + G::TW) {  // carried state of the next call
    const int rl = static_cast<int>(a.n_dec - 1 - jd0);
    float* co = a.carry_out + T.ch * kWbfmCarry;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (R * l + r == rl) {
        co[4] = d[r].x;
        co[5] = d[r].y;
        co[6] = 0.0f;
        co[7] = 0.0f;
      }
#pragma unroll
    for (int t2 = 0; t2 < kWbfmHist / 64; ++t2) {
      const int t = l + 64 * t2;
      a.hist_out[T.ch * kWbfmHist + t] = load_hist(T.xc, a.n, T.hc, kWbfmHist, a.n - kWbfmHist + t);
    }
  }
}

// ---- front tile, four-group decimator (k_wbfm_seg4) ------------------------------
// fu_tile's polyphase FIR with EIGHT outputs per lane instead of two. The 64 lanes
// are the four ds_read_b128 lane groups of gfx950 (A = {0-3, 12-15, 20-27},
// B = {4-11, 16-19, 28-31}, C, D = A, B + 32); group g sums phases 2g and 2g+1 for
// outputs 8l'..8l'+7 (l' = l & 15), and two permlane swaps (rows 0<->1, 2<->3, then
// the halves) add the four partial sums, leaving every lane two outputs. Per lane
// and tile: 24 window + 8 tap ds_read_b128 (fu_tile: 72 window reads), eight
// independent FMA chains per phase (fu_tile: two). Image rows carry one 16-B pad
// after every four chunks, so lane windows start 5 chunks apart and the 16 lanes
// of a read group hit 16 distinct bank quads; the pitch (91 chunks, odd) spreads
// the phase-scattered b64 staging stores.
#ifndef ORION_SEG4_PHASE_UNROLL
#define ORION_SEG4_PHASE_UNROLL 1
#endif
namespace g8 {
constexpr int PCH = 91;          // row pitch, 16-B chunks
constexpr int LRS = 2 * PCH;     // row pitch, f2 slots
constexpr int LDS_F2 = M * LRS;  // 11648 B
__host__ __device__ constexpr int pchunk(int c) { return 5 * (c >> 2) + (c & 3); }
__host__ __device__ constexpr int slot(int i) { return 2 * pchunk(i >> 1) + (i & 1); }
static_assert(slot(fu::G::TW + Q) < LRS && pchunk(fu::G::TW / 2) == 80, "row geometry");
__device__ __forceinline__ int group(int l) {
  const int i = l & 31;
  const bool a = i < 4 || (i >= 12 && i < 16) || (i >= 20 && i < 28);
  return (l >> 5) * 2 + (a ? 0 : 1);
}
// the lane holding the output before this lane's first one (lane 0: the carry)
__device__ __forceinline__ int prev_lane(int l) {
  const int row = l >> 4, lp = l & 15;
  return row == 0 ? 47 + lp : row == 2 ? lp : row == 1 ? 32 + lp : 16 + lp;
}
// this lane's first output (tile-relative): rows 0, 2, 1, 3 own 8l' + {0,1}, {2,3}, {4,5}, {6,7}
__device__ __forceinline__ int first_out(int l) {
  const int row = l >> 4;
  return 8 * (l & 15) + 2 * (row == 0 ? 0 : row == 2 ? 1 : row == 1 ? 2 : 3);
}
// One phase c of a lane's eight outputs: 12 window + 4 tap ds_read_b128 and 128
// v_pk_fma_f32. FIRST: the chains start with a product (d need not be zeroed).
// ORD: taps read first and the taps walked from q = Q-1 down, so the first FMAs
// need only the first window reads (entries 1..8) rather than the last.
template <bool FIRST, bool ORD>
__device__ __forceinline__ void phase(const f2* __restrict__ U, int c, int lp, const float* __restrict__ Gt,
                                      f2 (&d)[8]) {
  const f4* __restrict__ row = reinterpret_cast<const f4*>(U + c * LRS) + 5 * lp;
  const f4* __restrict__ tq = reinterpret_cast<const f4*>(Gt + c * Q);
  f4 w[12];
  float t[Q];
  if constexpr (ORD) {
#pragma unroll
    for (int q4 = Q / 4 - 1; q4 >= 0; --q4) {
      const f4 u = tq[q4];
      t[4 * q4] = u.x;
      t[4 * q4 + 1] = u.y;
      t[4 * q4 + 2] = u.z;
      t[4 * q4 + 3] = u.w;
    }
#pragma unroll
    for (int h = 0; h < 12; ++h) w[h] = row[5 * (h >> 2) + (h & 3)];
  } else {
#pragma unroll
    for (int h = 0; h < 12; ++h) w[h] = row[5 * (h >> 2) + (h & 3)];
#pragma unroll
    for (int q4 = 0; q4 < Q / 4; ++q4) {
      const f4 u = tq[q4];
      t[4 * q4] = u.x;
      t[4 * q4 + 1] = u.y;
      t[4 * q4 + 2] = u.z;
      t[4 * q4 + 3] = u.w;
    }
  }
#pragma unroll
  for (int qi = 0; qi < Q; ++qi) {
    const int q = ORD ? Q - 1 - qi : qi;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int m = r + Q - q;  // window entry 1 .. 23 (tap q of output 8l' + r)
      const f4& wc = w[m >> 1];
      const f2 xv = (m & 1) ? f2{wc.z, wc.w} : f2{wc.x, wc.y};
      if (FIRST && qi == 0) d[r] = splat2(t[q]) * xv;
      else d[r] = fma2(splat2(t[q]), xv, d[r]);
    }
  }
}
}  // namespace g8

template <bool A16, bool CLAMP, int X>
__device__ __forceinline__ void fu_tile8(const FuTile& T, int n, long long porg, long long jd0,
                                         const f2 (&ph)[8][2], f2 (&v)[8][2], const FuPrefetch& pf, f2 Sv,
                                         f2& carry, float* __restrict__ phit, int svi) {
  using G = fu::G;
  f2* __restrict__ U = T.U;
  const int l = T.l;
  if (n > 0) {  // halo: entries TW .. TW+Q of every row -> 0 .. Q, times e^{-j theta NEW}
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      const int e = l + 64 * r2;
      if (e < 72) {
        const int c = e / 9, h = e - 9 * c;
        const int dst = c * g8::LRS + 2 * g8::pchunk(h);
        const f4 w = *reinterpret_cast<const f4*>(U + dst + 2 * 80);  // pchunk(TW/2 + h) = 80 + pchunk(h)
        const f2 y0 = cmul(f2{w.x, w.y}, T.corr), y1 = cmul(f2{w.z, w.w}, T.corr);
        *reinterpret_cast<f4*>(U + dst) = f4{y0.x, y0.y, y1.x, y1.y};
      }
    }
    wave_lds_fence();
  }
  const bool bnd = porg < 0 || porg + 8LL * (G::TW + Q) > T.a.n;
#pragma unroll
  for (int k = 0; k < G::KL; ++k) {  // entry i + 16k = slot(i) + 20k
    U[T.s0 + 20 * k] = cmul_rot_pk(v[k][0], ph[k][0]);
    U[T.s1 + 20 * k] = cmul_rot_pk(v[k][1], ph[k][1]);
    if (k % 4 == 3) asm volatile("" ::: "memory");
  }
  asm volatile("" ::: "memory");
  front2_load<2, A16, CLAMP>(pf.xl, pf.nl, pf.porg, l, v);  // unconditional (see fu_tile)
  if (bnd) {
    wave_lds_fence();
#pragma unroll 1
    for (int p = (n == 0 ? 0 : 8 * Q) + l; p < 8 * (G::TW + Q); p += 64) {
      const long long Pp = porg + p;
      if (!CLAMP || Pp < 0 || Pp >= T.a.n || p < 8 * Q) {
        const int c = (-p) & 7;
        U[c * g8::LRS + g8::slot((p + c) / 8)] = cmul_rot(load_hist(T.xc, T.a.n, T.hc, kWbfmHist, Pp), T.tabc[p]);
      }
    }
  }
  wave_lds_fence();
  // group g: phases 2g, 2g+1; window entries 8l' .. 8l'+23 of the phase's row
  const int g = g8::group(l), lp = l & 15;
  f2 d[8];
  if constexpr ((X & 1) != 0) {
    // phase 2g opens the eight chains with a product (no zeroing), phase 2g+1
    // follows; the barrier keeps the second phase's reads behind the first's FMAs
    g8::phase<true, (X & 2) != 0>(U, 2 * g, lp, T.Gt, d);
    asm volatile("" ::: "memory");
    g8::phase<false, (X & 2) != 0>(U, 2 * g + 1, lp, T.Gt, d);
  } else {
#pragma unroll
  for (int r = 0; r < 8; ++r) d[r] = f2{0.0f, 0.0f};
#pragma unroll ORION_SEG4_PHASE_UNROLL
  for (int s = 0; s < 2; ++s) {
    const int c = 2 * g + s;
    const f4* __restrict__ row = reinterpret_cast<const f4*>(U + c * g8::LRS) + 5 * lp;
    f4 w[12];
#pragma unroll
    for (int h = 0; h < 12; ++h) w[h] = row[5 * (h >> 2) + (h & 3)];
    const f4* __restrict__ tq = reinterpret_cast<const f4*>(T.Gt + c * Q);
    float t[Q];
#pragma unroll
    for (int q4 = 0; q4 < Q / 4; ++q4) {
      const f4 u = tq[q4];
      t[4 * q4] = u.x;
      t[4 * q4 + 1] = u.y;
      t[4 * q4 + 2] = u.z;
      t[4 * q4 + 3] = u.w;
    }
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int m = r + Q - q;  // window entry 1 .. 23 (tap q of output 8l' + r)
        const f4& wc = w[m >> 1];
        d[r] = fma2(splat2(t[q]), (m & 1) ? f2{wc.z, wc.w} : f2{wc.x, wc.y}, d[r]);
      }
  }
  }
  // rows 0<->1, 2<->3: even rows keep outputs 0..3, odd rows 4..7 (x: d[i], y: d[i+4])
  f2 K[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const auto sx = __builtin_amdgcn_permlane16_swap(__float_as_uint(d[i].x), __float_as_uint(d[i + 4].x), false, false);
    const auto sy = __builtin_amdgcn_permlane16_swap(__float_as_uint(d[i].y), __float_as_uint(d[i + 4].y), false, false);
    K[i] = f2{__uint_as_float(sx[0]), __uint_as_float(sy[0])} + f2{__uint_as_float(sx[1]), __uint_as_float(sy[1])};
  }
  // halves: rows 0, 1 keep K[0..1], rows 2, 3 K[2..3]
  f2 F[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const auto sx = __builtin_amdgcn_permlane32_swap(__float_as_uint(K[i].x), __float_as_uint(K[i + 2].x), false, false);
    const auto sy = __builtin_amdgcn_permlane32_swap(__float_as_uint(K[i].y), __float_as_uint(K[i + 2].y), false, false);
    F[i] = f2{__uint_as_float(sx[0]), __uint_as_float(sy[0])} + f2{__uint_as_float(sx[1]), __uint_as_float(sy[1])};
  }
  const f2 S = f2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(Sv.x), svi)),
                  __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Sv.y), svi))};
  F[0] = cmul(F[0], S);
  F[1] = cmul(F[1], S);
  if (n == 0 && !T.first) {  // d[A-1] from this tile's image (as fu_tile)
    f2 acc = f2{0.0f, 0.0f};
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2) {
      const int k = 2 * l + t2, c = k & 7, q = k >> 3;
      acc = fma2(splat2(T.Gt[c * Q + q]), U[c * g8::LRS + g8::slot(15 - q)], acc);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
      acc += f2{__shfl_xor(acc.x, off, 64), __shfl_xor(acc.y, off, 64)};
    carry = cmul(acc, S);
  }
  const int src = g8::prev_lane(l);
  f2 pv = f2{__shfl(F[1].x, src, 64), __shfl(F[1].y, src, 64)};
  if (l == 0) pv = carry;
  const int j0 = g8::first_out(l);
  *reinterpret_cast<f2*>(phit + j0) = f2{fm_disc_pk_rcp(F[0], pv, T.C.k), fm_disc_pk_rcp(F[1], F[0], T.C.k)};
  carry = f2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(F[1].x), 63)),
             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(F[1].y), 63))};
  const WbfmArgs& a = T.a;
  if (jd0 <= a.n_dec - 1 && a.n_dec - 1 < jd0 + G::TW) {  // carried state of the next call
    const int rl = static_cast<int>(a.n_dec - 1 - jd0);
    float* co = a.carry_out + T.ch * kWbfmCarry;
#pragma unroll
    for (int r = 0; r < 2; ++r)
      if (j0 + r == rl) {
        co[4] = F[r].x;
        co[5] = F[r].y;
        co[6] = 0.0f;
        co[7] = 0.0f;
      }
#pragma unroll
    for (int t2 = 0; t2 < kWbfmHist / 64; ++t2) {
      const int t = l + 64 * t2;
      a.hist_out[T.ch * kWbfmHist + t] = load_hist(T.xc, a.n, T.hc, kWbfmHist, a.n - kWbfmHist + t);
    }
  }
}

// Range geometry shared by the front and the back of one range.
struct FuRange {
  int r, ch, wl;
  long long A, B;
  int Lr;
  bool first, last;
};
template <int N>
__device__ __forceinline__ FuRange fu_range(const WbfmArgs& a, int r, int wpc) {
  FuRange g;
  g.r = r;
  g.ch = r / wpc;
  g.wl = r - g.ch * wpc;
  g.A = static_cast<long long>(g.wl) * fu::Geo<N>::L;
  g.B = min(g.A + fu::Geo<N>::L, a.n_dec);
  g.Lr = static_cast<int>(g.B - g.A);
  g.first = g.wl == 0;
  g.last = g.B == a.n_dec;
  return g;
}

// Where range g's first tile starts (its first two tiles are prefetched into va/vb).
__device__ __forceinline__ FuPrefetch fu_origin(const WbfmArgs& a, const FuRange& g) {
  const bool tiny = a.n < 2;
  FuPrefetch p;
  p.xl = tiny ? a.hist_in + g.ch * kWbfmHist : a.x + g.ch * a.x_stride;
  p.nl = tiny ? kWbfmHist : a.n;
  p.porg = 8LL * (g.A - Q);
  p.on = true;
  return p;
}

// The front of one range: N tiles -> Phi[0 .. L); dA = d[A] (for phi[A]) and
// dlast = d[A+L-1] (for the next range). On entry va/vb hold the range's first
// two tiles; on exit, when nx.on, the next range's first two (nx = its origin).
template <int N, bool A16, bool CLAMP>
__device__ __forceinline__ void fu_front_range(const WbfmArgs& a, const WbfmFrontConst& C, const FuRange& g,
                                               f2* U, float* Phi, const float* Gt, f2 (&va)[8][2], f2 (&vb)[8][2],
                                               const FuPrefetch& nx, f2& dA, f2& dlast) {
  using G = fu::G;
  const int l = threadIdx.x & 63;
  const f2* __restrict__ tabc = a.tab + static_cast<long long>(g.ch) * kWbfmNS;
  const f2* __restrict__ xc = a.x + g.ch * a.x_stride;
  const f2* __restrict__ hc = a.hist_in + g.ch * kWbfmHist;
  const FuPrefetch org = fu_origin(a, g);
  const f4 tv = *reinterpret_cast<const f4*>(tabc + 8 * Q + 2 * l);
  const f2 tb0 = f2{tv.x, tv.y}, tb1 = f2{tv.z, tv.w};
  f2 ph[G::KL][2];
#pragma unroll
  for (int k = 0; k < G::KL; ++k) {
    const f2 ek = tabc[128 * k];
    ph[k][0] = cmul(tb0, ek);
    ph[k][1] = cmul(tb1, ek);
  }
  const f2 cn = tabc[G::NEW];
  const int c0 = (-2 * l) & 7, c1 = (-2 * l - 1) & 7;
  const FuTile T{a, C, U, Phi, Gt, xc, hc, tabc, g.ch, l, c0 * G::LR + (8 * Q + 2 * l + c0) / 8,
                 c1 * G::LR + (8 * Q + 2 * l + 1 + c1) / 8, f2{cn.x, -cn.y}, g.first};
  long long porg = org.porg;  // tile n computes d[A + 128 n + (0..127)]
  {  // halo rows of the first tile (p = 2l, 2l+1): clamped here, exact via the boundary fixup
    const long long P0 = porg + 2 * l;
    const long long hi = (org.nl & ~1LL) - 2;
    const long long Pc = P0 < 0 ? 0 : (P0 > hi ? hi : P0);
    const f2 x0 = org.xl[Pc], x1 = org.xl[Pc + 1];
    const f4 th = *reinterpret_cast<const f4*>(tabc + 2 * l);
    U[c0 * G::LR + (2 * l + c0) / 8] = cmul_rot(x0, f2{th.x, th.y});
    U[c1 * G::LR + (2 * l + 1 + c1) / 8] = cmul_rot(x1, f2{th.z, th.w});
  }
  {  // p = -l (row c = l, i = 0), l = 1..7: used only by d[A-1]. Not the first
     // range, so porg - l >= 0: a plain load (a branchy one would drain the prefetch)
    const long long Pm = max(porg - (l & 7), 0LL);
    const f2 xm = xc[Pm];
    const f2 tc = tabc[l & 7];
    if (!g.first && l >= 1 && l < 8) U[l * G::LR] = cmul_rot(xm, f2{tc.x, -tc.y});
  }
  const f2 Sv = phasor_q64(static_cast<uint64_t>(a.k0 + porg + 1 + static_cast<long long>(l) * G::NEW),
                           a.step[g.ch]);
  f2 carry = f2{0.0f, 0.0f};
  if (g.first) {  // d[-1]: the last decimated sample of the previous call (fm.rs:29 on reset)
    const float* ci = a.carry_in + g.ch * kWbfmCarry;
    carry = f2{ci[4], ci[5]};
  }
#pragma unroll 1
  for (int n = 0; n < N; n += 2, porg += 2 * G::NEW) {
    const long long jd0 = g.A + static_cast<long long>(n) * G::TW;
    FuPrefetch p0{org.xl, org.nl, porg + 2 * G::NEW, true}, p1{org.xl, org.nl, porg + 3 * G::NEW, true};
    // past the range: the next range's first tiles, or (none) a dummy read of the
    // channel's first tile, shared by all of the channel's ranges so that it hits
    // in L2 (re-reading this range's own tile would cost HBM: 2 tiles in N)
    const FuPrefetch dummy{org.xl, org.nl, -8LL * Q, true};
    if (n + 2 >= N) p0 = nx.on ? FuPrefetch{nx.xl, nx.nl, nx.porg, true} : dummy;
    if (n + 3 >= N) p1 = nx.on ? FuPrefetch{nx.xl, nx.nl, nx.porg + G::NEW, true} : dummy;
    fu_tile<A16, CLAMP>(T, n, porg, jd0, PhArr{ph}, va, p0, Sv, carry, dA, T.Phi + G::TW * n, n);
    fu_tile<A16, CLAMP>(T, n + 1, porg + G::NEW, jd0 + G::TW, PhArr{ph}, vb, p1, Sv, carry, dA, T.Phi + G::TW * (n + 1),
                        n + 1);
  }
  dlast = carry;
}

// The back of one range (LpCascade, audio FIR) from Phi[0 .. L), with one
// hand-off to the next range that depends on nothing but this range's phi:
//  - the zero-state pass gives every chunk's zero-state entering state and the
//    range's zero-state end state a_w. The true state entering range w+1 is
//    a_w + A^L (true state entering w) = a_w, since ||A^L|| is negligible (the
//    host checks it);
//  - the last 128 IIR outputs of this range (the next range's FIR history) are
//    the zero-state recurrence over them: their true values differ by A^{L-128}
//    times the entering state, also negligible;
// so both are published right after the zero-state pass, and a range waits only
// for its predecessor's zero-state pass (no wait chain). P is this wave's
// pair-image region (may alias Phi: Phi is read into registers first).
template <int N>
__device__ __forceinline__ void fu_back_range(const WbfmArgs& a, const WbfmFrontConst& C, const WbfmFusedConst& Bc,
                                              const FuRange& g, float* Phi, f2* P) {
  using Y = fu::Geo<N>;
  constexpr int L = Y::L, NH = Y::NH, CH = Y::CH;
  constexpr int TL = 64 - fu::PB / CH;  // first lane whose half-B chunk lies in the last 128
  const int l = threadIdx.x & 63;
  const int ch = g.ch;
  const long long A = g.A;
  const int Lr = g.Lr;
  const bool first = g.first, last = g.last;
  uint32_t* slot = a.hand + static_cast<long long>(g.r) * kFuSlot;
  const uint32_t* pslot_ = a.hand + static_cast<long long>(g.r - 1) * kFuSlot;
  uint32_t* flag = a.flags + 3LL * g.r;
  const uint32_t* pflag = a.flags + 3LL * (g.r - 1);
  const float* __restrict__ ci = a.carry_in + ch * kWbfmCarry;

  // ==== zero-state pass, f64 scan per half ====
  const Biquad2 bq{splat2(Bc.b0), splat2(Bc.b1), splat2(Bc.b2), splat2(Bc.a1), splat2(Bc.a2)};
  f2 xs[CH];
#pragma unroll
  for (int i = 0; i < CH; i += 4) {
    const f4 u = *reinterpret_cast<const f4*>(Phi + CH * l + i);
    const f4 w = *reinterpret_cast<const f4*>(Phi + NH + CH * l + i);
    xs[i] = f2{u.x, w.x};
    xs[i + 1] = f2{u.y, w.y};
    xs[i + 2] = f2{u.z, w.z};
    xs[i + 3] = f2{u.w, w.w};
  }
  wave_lds_fence();
  f2 s[4] = {f2{0, 0}, f2{0, 0}, f2{0, 0}, f2{0, 0}};
#pragma unroll
  for (int i = 0; i < CH; ++i) (void)bq.lp4(s, xs[i]);
  double q[2][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    q[0][k] = s[k].x;
    q[1][k] = s[k].y;
  }
#pragma unroll 1
  for (int st = 0; st < 6; ++st) {
    const int dd = 1 << st;
    double o[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < 4; ++k) o[h][k] = __shfl_up(q[h][k], dd, 64);
    if (l >= dd) {
      matvec_acc<4>(Bc.pw + st * 16, o[0], q[0]);
      matvec_acc<4>(Bc.pw + st * 16, o[1], q[1]);
    }
  }
  // zero-state entering states (range-relative): half A lane l: exclusive prefix
  // A; half B lane l: A^{CH l} aggA + exclusive prefix B
  double aggA[4], agg[4], ez[2][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    aggA[k] = __shfl(q[0][k], 63, 64);
    agg[k] = __shfl(q[1][k], 63, 64);
  }
  matvec_acc<4>(Bc.mh, aggA, agg);  // zero-state end state of the range
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double o = __shfl_up(q[h][k], 1, 64);
      ez[h][k] = l == 0 ? 0.0 : o;
    }
  matvec_acc<4>(a.lanemats_fu + l * 16, aggA, ez[1]);
  fu::trace(a, g.r, 2);

  // ==== hand-off: publish (end state, last 128 outputs), then take the predecessor's ====
  if (!last) {
    f2 e[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = f2{0.0f, static_cast<float>(ez[1][k])};
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const f2 f = bq.lp4(e, xs[i]);  // half B (.y): the range's last CH*64 outputs
      if (l >= TL) fu::st_agent(slot + 16 + (l - TL) * CH + i, __float_as_uint(f.y));
    }
    if (l < 8) {
      const int kk = l >> 1;
      const double v8 = kk == 0 ? agg[0] : kk == 1 ? agg[1] : kk == 2 ? agg[2] : agg[3];
      const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v8));
      fu::st_agent(slot + 2 + l, (l & 1) ? static_cast<uint32_t>(b >> 32) : static_cast<uint32_t>(b));
    }
    fu::publish(flag + 0, a.epoch, l);
  }
  double sw[4];
  float hist[2];  // f[t - 128], t = l, l + 64: this range's FIR history
  if (first) {
#pragma unroll
    for (int k = 0; k < 4; ++k) sw[k] = ci[k];
    hist[0] = ci[8 + l];
    hist[1] = ci[8 + 64 + l];
  } else {
    fu::wait_for(pflag + 0, a.epoch, a.err);
#pragma unroll
    for (int k = 0; k < 4; ++k) sw[k] = fu::u2d(fu::ld_agent(pslot_ + 2 + 2 * k), fu::ld_agent(pslot_ + 3 + 2 * k));
    hist[0] = __uint_as_float(fu::ld_agent(pslot_ + 16 + l));
    hist[1] = __uint_as_float(fu::ld_agent(pslot_ + 16 + 64 + l));
  }
  fu::trace(a, g.r, 3);
  // true entering states: zero-state ones plus the entering state's propagation,
  // half A: A^{CH l} sw; half B: A^{CH l} A^NH sw
  f2 ef[4];
  {
    double sB[4] = {0, 0, 0, 0};
    matvec_acc<4>(Bc.mh, sw, sB);
    matvec_acc<4>(a.lanemats_fu + l * 16, sw, ez[0]);
    matvec_acc<4>(a.lanemats_fu + l * 16, sB, ez[1]);
#pragma unroll
    for (int k = 0; k < 4; ++k) ef[k] = f2{static_cast<float>(ez[0][k]), static_cast<float>(ez[1][k])};
  }

  // ==== pass 2 (reference recurrence) -> P[j] = (f[j], f[j+NH]) ====
  {
    const int jl = Lr - 1;  // local index of the channel's last sample (last range)
    float cap[4] = {0, 0, 0, 0};
    bool have = false;
    // pslot(CH l + PB + i) = pslot(CH l + PB) + i for i < CH: one base address (the
    // per-i form is not seen as linear and its eight addresses spill to scratch,
    // whose reloads wait vmcnt(0) on the prefetched tiles)
    int po = Y::pslot(CH * l + fu::PB);
    asm volatile("" : "+v"(po));  // not hoisted out of the sub-range loop (see iir16's pass 2)
    f2* __restrict__ pb = P + po;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int j = CH * l + i;
      const f2 f = bq.lp4(ef, xs[i]);
      pb[i] = f;
      if (last) {
        if (j == jl) {
#pragma unroll
          for (int k = 0; k < 4; ++k) cap[k] = ef[k].x;
          have = true;
        }
        if (j + NH == jl) {
#pragma unroll
          for (int k = 0; k < 4; ++k) cap[k] = ef[k].y;
          have = true;
        }
      }
    }
    if (have) {
      float* co = a.carry_out + ch * kWbfmCarry;
#pragma unroll
      for (int k = 0; k < 4; ++k) co[k] = cap[k];
    }
  }
  wave_lds_fence();
  // pairs j in [-128, 0): .x = the FIR history, .y = f[j + NH] (this range's own)
#pragma unroll
  for (int r2 = 0; r2 < 2; ++r2) {
    const int t = l + 64 * r2;  // j = t - 128
    P[Y::pslot(t)] = f2{hist[r2], P[Y::pslot(t + NH)].x};
  }
  wave_lds_fence();
  fu::trace(a, g.r, 4);

  // ==== audio FIR (fir.rs:57-66) over [A, B) ====
  // lane l: outputs j = CH l + i and j + NH (i < CH); tap k = 16 kb + kk of
  // output i reads f[j - k]: window m = i + 15 - kk of the CH+15 pairs from
  // e = CH l - 16 kb - 15 + 128 = CH (l - 16kb/CH) + 113; slot = (CH+1)(l -
  // 16kb/CH) + 113 + m + (113 + m)/CH: a per-lane base and compile-time offsets.
  {
    constexpr int KA = 128;
    f2 acc[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) acc[i] = f2{0.0f, 0.0f};
#pragma unroll 1
    for (int kb = 0; kb < KA / 16; ++kb) {
      const f2* __restrict__ Pl = P + (CH + 1) * (l - 16 * kb / CH) + 113;
      f2 w[CH + 15];
#pragma unroll
      for (int m = 0; m < CH + 15; ++m) w[m] = Pl[m + (113 + m) / CH];
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const f2 tap = splat2(Bc.a[16 * kb + kk]);
#pragma unroll
        for (int i = 0; i < CH; ++i) acc[i] = fma2(tap, w[i + 15 - kk], acc[i]);
      }
    }
    float* __restrict__ y = a.y + ch * a.y_stride + A;
    if (Lr == L && (reinterpret_cast<uintptr_t>(y) & 15) == 0) {
      float4* ya = reinterpret_cast<float4*>(y + CH * l);
      float4* yb = reinterpret_cast<float4*>(y + NH + CH * l);
#pragma unroll
      for (int i = 0; i < CH; i += 4) {
        ya[i / 4] = float4{acc[i].x, acc[i + 1].x, acc[i + 2].x, acc[i + 3].x};
        yb[i / 4] = float4{acc[i].y, acc[i + 1].y, acc[i + 2].y, acc[i + 3].y};
      }
    } else {
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int j = CH * l + i;
        if (j < Lr) y[j] = acc[i].x;
        if (j + NH < Lr) y[j + NH] = acc[i].y;
      }
    }
  }
  fu::trace(a, g.r, 5);
  if (last) {  // the next call's FIR history: f[n_dec - 128 .. n_dec)
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      const int t = l + 64 * r2;
      const int j = Lr - 128 + t;  // >= -128
      const float f = j < NH ? P[Y::pslot(j + fu::PB)].x : P[Y::pslot(j - NH + fu::PB)].y;
      a.carry_out[ch * kWbfmCarry + 8 + t] = f;
    }
  }
  wave_lds_fence();  // P / Phi reads done before the caller reuses them
}

// Single-role form: one wave per range (front, then back).
template <int N, bool A16, bool CLAMP, bool PERS>
__global__ __launch_bounds__(64, fu::Geo<N>::WavesPerSimd) void k_wbfm_fused(const WbfmArgs a,
                                                                             const WbfmFrontConst C,
                                                                             const WbfmFusedConst Bc, int wpc,
                                                                             int total) {
  using G = fu::G;
  using Y = fu::Geo<N>;
  __shared__ __attribute__((aligned(16))) unsigned char lds[Y::LdsBytes];
  __shared__ __attribute__((aligned(16))) float Gt[128];
  f2* U = reinterpret_cast<f2*>(lds);                          // front image ...
  float* Phi = reinterpret_cast<float*>(lds + G::LDS_F2 * 8);  // ... and phi, then
  f2* P = reinterpret_cast<f2*>(lds);                          // the FIR pairs over both
  Gt[threadIdx.x] = C.g[threadIdx.x];
  Gt[threadIdx.x + 64] = C.g[threadIdx.x + 64];
  f2 va[G::KL][2], vb[G::KL][2];
  f2 dA = f2{0, 0}, dlast = f2{0, 0};
  if constexpr (!PERS) {  // one range per wave (gridDim.x = total)
    const FuRange g = fu_range<N>(a, blockIdx.x, wpc);
    fu::trace(a, g.r, 0);
    const FuPrefetch org = fu_origin(a, g);
    front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg, threadIdx.x, va);
    front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg + G::NEW, threadIdx.x, vb);
    fu_front_range<N, A16, CLAMP>(a, C, g, U, Phi, Gt, va, vb, FuPrefetch{nullptr, 0, 0, false}, dA, dlast);
    fu::trace(a, g.r, 1);
    if (a.fu_abl & 1) {  // timing only: front alone (phi kept alive)
      if (Phi[threadIdx.x] == 1234.5f) a.y[threadIdx.x] = Phi[threadIdx.x];
      return;
    }
    fu_back_range<N>(a, C, Bc, g, Phi, P);
  } else {
    // persistent (gridDim.x <= resident capacity): ranges r = blockIdx.x + k
    // gridDim.x, each range's first two tiles prefetched across the previous
    // range's back phase
    int r = blockIdx.x;
    const FuPrefetch org = fu_origin(a, fu_range<N>(a, r, wpc));
    front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg, threadIdx.x, va);
    front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg + G::NEW, threadIdx.x, vb);
#pragma unroll 1
    for (; r < total; r += gridDim.x) {
      const FuRange g = fu_range<N>(a, r, wpc);
      fu::trace(a, g.r, 0);
      const int rn = r + static_cast<int>(gridDim.x);
      const FuPrefetch nx = rn < total ? fu_origin(a, fu_range<N>(a, rn, wpc)) : FuPrefetch{nullptr, 0, 0, false};
      fu_front_range<N, A16, CLAMP>(a, C, g, U, Phi, Gt, va, vb, nx, dA, dlast);
      fu::trace(a, g.r, 1);
      if (a.fu_abl & 1) {
        if (Phi[threadIdx.x] == 1234.5f) a.y[threadIdx.x] = Phi[threadIdx.x];
        wave_lds_fence();
        continue;
      }
      fu_back_range<N>(a, C, Bc, g, Phi, P);
    }
  }
}

// ---- segmented chain -----------------------------------------------------------
// k_wbfm_seg: the whole chain in one kernel, ONE round of waves (the grid is the
// resident capacity, so no wave waits for a slot) and the back of the chain
// interleaved with the input stream. One wave per segment of S decimated outputs
// [A, B) of a channel (S a multiple of the sub-range, L = 1024), walked in front
// tiles of 128 outputs with the input prefetched two tiles ahead. Every 8 tiles
// a sub-range is complete and its back runs right there (LpCascade, audio FIR,
// stores) while the two prefetched tiles are in flight, so the input stream
// pauses for one sub-range's back at most instead of a whole range's:
//   sub-range 0:  zero-state pass only (its entering state is the predecessor
//                 segment's END state, not known yet). It yields the zero-state
//                 end state and the zero-state last 128 IIR outputs, which are
//                 the true ones to f32 resolution: the host selects this kernel
//                 only when ||A^896|| is negligible (the predecessor's state has
//                 decayed by then; ~1e-16 for the WBFM defaults);
//   sub-range k>0: full back from the previous sub-range's exact f32 end state
//                 and last 128 IIR outputs (the FIR history), both carried in
//                 registers; the last one publishes the segment's end state and
//                 tail to its successor;
//   end:          wait for the predecessor's end state and tail (published at
//                 its last sub-range: waves of one round finish together, and no
//                 wait chain forms), then sub-range 0's back from them.
// A segment of one sub-range publishes its zero-state end state and tail at once.
#ifndef ORION_SEG_PRIO
#define ORION_SEG_PRIO 1
#endif
#ifndef ORION_SEG_ABL
#define ORION_SEG_ABL 0  // timing experiments only (separate builds): 1 no sub-range backs, 2 no
                         // zero-state pass, 4 no deferred back, 8 no spread FIR blocks (seg2)
#endif
#ifndef ORION_SEG_EARLY_PUB
#define ORION_SEG_EARLY_PUB 1  // k_wbfm_seg publishes a segment's end state before its last audio FIR
#endif
#ifndef ORION_SEG_BACK_KB
#define ORION_SEG_BACK_KB 8  // audio FIR taps per block in k_wbfm_seg's sub-range back
#endif
#ifndef ORION_SEG_BACK_UNROLL
#define ORION_SEG_BACK_UNROLL 1
#endif
#ifndef ORION_SEG_PRIO_Q16
#define ORION_SEG_PRIO_Q16 9
#endif
constexpr bool kSegPrio = ORION_SEG_PRIO;
constexpr int kSegPrioQ16 = ORION_SEG_PRIO_Q16;  // late waves lead for this many 16ths of their tiles
namespace sg {
constexpr int NS = 8;          // front tiles per sub-range
using Y = fu::Geo<NS>;         // L 1024, NH 512, CH 8
constexpr int L = Y::L;
constexpr int CH = Y::CH;
constexpr int WBytes = (Y::PSlots * 8 > L * 4) ? Y::PSlots * 8 : L * 4;

__device__ __forceinline__ double uni(double v) {  // wave-uniform value -> SGPRs
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane(static_cast<int>(b));
  const int hi = __builtin_amdgcn_readfirstlane(static_cast<int>(b >> 32));
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// Zero-state LpCascade pass over one sub-range's phi: xs = the lane's two chunks
// (half A, half B as a float2), ez = zero-state entering state of each chunk
// (range-relative), agg = zero-state end state of the sub-range.
__device__ __forceinline__ void zero_state(const WbfmFusedConst& Bc, const double* __restrict__ lm,
                                           const float* __restrict__ Phi, int l, f2 (&xs)[CH],
                                           double (&ez)[2][4], double (&agg)[4]) {
  constexpr int NH = Y::NH;
  const Biquad2 bq{splat2(Bc.b0), splat2(Bc.b1), splat2(Bc.b2), splat2(Bc.a1), splat2(Bc.a2)};
#pragma unroll
  for (int i = 0; i < CH; i += 4) {
    const f4 u = *reinterpret_cast<const f4*>(Phi + CH * l + i);
    const f4 w = *reinterpret_cast<const f4*>(Phi + NH + CH * l + i);
    xs[i] = f2{u.x, w.x};
    xs[i + 1] = f2{u.y, w.y};
    xs[i + 2] = f2{u.z, w.z};
    xs[i + 3] = f2{u.w, w.w};
  }
  wave_lds_fence();
  f2 s[4] = {f2{0, 0}, f2{0, 0}, f2{0, 0}, f2{0, 0}};
#pragma unroll
  for (int i = 0; i < CH; ++i) (void)bq.lp4(s, xs[i]);
  double q[2][4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    q[0][k] = s[k].x;
    q[1][k] = s[k].y;
  }
#pragma unroll 1
  for (int st = 0; st < 6; ++st) {
    const int dd = 1 << st;
    double o[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < 4; ++k) o[h][k] = __shfl_up(q[h][k], dd, 64);
    if (l >= dd) {
      matvec_acc<4>(Bc.pw + st * 16, o[0], q[0]);
      matvec_acc<4>(Bc.pw + st * 16, o[1], q[1]);
    }
  }
  double aggA[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    aggA[k] = __shfl(q[0][k], 63, 64);
    agg[k] = __shfl(q[1][k], 63, 64);
  }
  matvec_acc<4>(Bc.mh, aggA, agg);
#pragma unroll
  for (int k = 0; k < 4; ++k) agg[k] = uni(agg[k]);
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double o = __shfl_up(q[h][k], 1, 64);
      ez[h][k] = l == 0 ? 0.0 : o;
    }
  matvec_acc<4>(lm + l * 16, aggA, ez[1]);
}

// Sub-range 0's first pass: zero-state end state sw and zero-state last 128 IIR
// outputs (hout[r] = f[L - 128 + l + 64 r]); tmp: 128 floats of free LDS.
__device__ __forceinline__ void zs_only(const WbfmFusedConst& Bc, const double* lm, const float* Phi, float* tmp,
                                        int l, double (&sw)[4], float (&hout)[2]) {
  constexpr int TL = 64 - fu::PB / CH;  // lanes whose half-B chunk lies in the last 128
  f2 xs[CH];
  double ez[2][4];
  zero_state(Bc, lm, Phi, l, xs, ez, sw);
  const Biquad2 bq{splat2(Bc.b0), splat2(Bc.b1), splat2(Bc.b2), splat2(Bc.a1), splat2(Bc.a2)};
  f2 e[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) e[k] = f2{0.0f, static_cast<float>(ez[1][k])};
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const f2 f = bq.lp4(e, xs[i]);
    if (l >= TL) tmp[(l - TL) * CH + i] = f.y;
  }
  wave_lds_fence();
  hout[0] = tmp[l];
  hout[1] = tmp[l + 64];
  wave_lds_fence();
}

// Sub-range IIR with lane l owning the 16 CONSECUTIVE samples 16l .. 16l+15: chunk E
// (16l .. 16l+7) in the x halves and chunk O (16l+8 .. 16l+15) in the y halves of
// xs, both zero-state passes packed. The lane aggregate A^8 zE + zO is scanned over
// the 64 lanes (Kogge-Stone, f64, step matrices A^(16 2^s) = pw[s+1], mh) with the
// entering state sw folded into lane 0, so the scan yields every lane's TRUE entering
// state directly: no per-lane transition matrices (lanemats) and half the f64 work
// of zero_state + the A^{CH l} products. ef: the f32 entering states of E and O;
// send: the f64 end state after sample L-1 (uniform).
static_assert(offsetof(WbfmFusedConst, mh) == offsetof(WbfmFusedConst, pw) + 6 * 16 * sizeof(double),
              "iir16 reads A^512 as pw[6]");
__device__ __forceinline__ void iir16(const WbfmFusedConst& Bc, const float* __restrict__ Phi, int l,
                                      const double (&sw)[4], f2 (&xs)[CH], f2 (&ef)[4], double (&send)[4]) {
#pragma unroll
  for (int i = 0; i < CH; i += 4) {
    const f4 u = *reinterpret_cast<const f4*>(Phi + 16 * l + i);
    const f4 w = *reinterpret_cast<const f4*>(Phi + 16 * l + 8 + i);
    xs[i] = f2{u.x, w.x};
    xs[i + 1] = f2{u.y, w.y};
    xs[i + 2] = f2{u.z, w.z};
    xs[i + 3] = f2{u.w, w.w};
  }
  wave_lds_fence();
  const Biquad2 bq{splat2(Bc.b0), splat2(Bc.b1), splat2(Bc.b2), splat2(Bc.a1), splat2(Bc.a2)};
  f2 z[4] = {f2{0, 0}, f2{0, 0}, f2{0, 0}, f2{0, 0}};
#pragma unroll
  for (int i = 0; i < CH; ++i) (void)bq.lp4(z, xs[i]);
  double zE[4], q[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    zE[k] = z[k].x;
    q[k] = z[k].y;
  }
  matvec_acc<4>(Bc.pw, zE, q);  // A^8 zE + zO
  {
    double f[4] = {0, 0, 0, 0};
    matvec_acc<4>(Bc.pw + 16, sw, f);  // A^16 sw
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] += l == 0 ? f[k] : 0.0;
  }
#pragma unroll 1
  for (int st = 0; st < 6; ++st) {
    const int dd = 1 << st;
    double o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = __shfl_up(q[k], dd, 64);
    if (l >= dd) matvec_acc<4>(Bc.pw + (st + 1) * 16, o, q);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long long b = __double_as_longlong(q[k]);
    const int lo = __builtin_amdgcn_readlane(static_cast<int>(b), 63);
    const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), 63);
    send[k] = __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
  }
  double eE[4], eO[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double o = __shfl_up(q[k], 1, 64);
    eE[k] = l == 0 ? sw[k] : o;
    eO[k] = zE[k];
  }
  matvec_acc<4>(Bc.pw, eE, eO);  // entering O = A^8 (entering E) + zE
#pragma unroll
  for (int k = 0; k < 4; ++k) ef[k] = f2{static_cast<float>(eE[k]), static_cast<float>(eO[k])};
}

// zs_only with iir16: sub-range 0's zero-state end state sw and zero-state last 128
// IIR outputs (lanes 56..63 run their pass 2; tmp: 128 floats of free LDS).
__device__ __forceinline__ void zs_only16(const WbfmFusedConst& Bc, const float* Phi, float* tmp, int l,
                                          double (&sw)[4], float (&hout)[2]) {
  const double zero[4] = {0, 0, 0, 0};
  f2 xs[CH], ef[4];
  iir16(Bc, Phi, l, zero, xs, ef, sw);
  const Biquad2 bq{splat2(Bc.b0), splat2(Bc.b1), splat2(Bc.b2), splat2(Bc.a1), splat2(Bc.a2)};
  int to = 16 * (l - 56);
  asm volatile("" : "+v"(to));  // not hoisted and spilled (see iir16's pass 2)
  float* __restrict__ tl = tmp + to;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const f2 f = bq.lp4(ef, xs[i]);
    if (l >= 56) {  // f[16l + i], f[16l + 8 + i]: tail index 16(l - 56) + i (+ 8)
      tl[i] = f.x;
      tl[8 + i] = f.y;
    }
  }
  wave_lds_fence();
  hout[0] = tmp[l];
  hout[1] = tmp[l + 64];
  wave_lds_fence();
}

// The back of one sub-range [A0, A0 + Lr) from its exact entering state sw and
// FIR history hist (f[A0 - 128 + l + 64 r]): pass 2 (the reference's f32
// recurrence) -> pair image P -> audio FIR -> y. Returns the end state (after
// f[A0 + L - 1]) in sw and this sub-range's last 128 IIR outputs in hist. P may
// alias Phi (Phi is read into registers first). chan_last: the channel's last
// sub-range (writes the IIR state and FIR history carried to the next call).
// publish_r >= 0: publish the end state and last 128 IIR outputs to the successor
// (publish_end) as soon as they are known, before the audio FIR.
__device__ __forceinline__ void publish_end(const WbfmArgs& a, int r, const double (&sw)[4], const float (&hist)[2],
                                            int l, int stride = kFuSlot);
template <int KB = ORION_SEG_BACK_KB, bool I16 = false>
__device__ __forceinline__ void back(const WbfmArgs& a, const WbfmFusedConst& Bc, int ch, long long A0, int Lr,
                                     bool chan_last, const float* Phi, f2* P, int l, double (&sw)[4],
                                     float (&hist)[2], int publish_r = -1, int stride = kFuSlot, int trace_r = -1) {
  constexpr int NH = Y::NH;
  const Biquad2 bq{splat2(Bc.b0), splat2(Bc.b1), splat2(Bc.b2), splat2(Bc.a1), splat2(Bc.a2)};
  f2 xs[CH];
  f2 ef[4];
  if constexpr (I16) {  // lane l: samples 16l .. 16l+15 (iir16), written to P one scalar at a time
    double send[4];
    iir16(Bc, Phi, l, sw, xs, ef, send);
    if (trace_r >= 0) fu::trace(a, trace_r, 10);
    const int jl = Lr - 1;
    float cap[4] = {0, 0, 0, 0};
    bool have = false;
    // f[16l + i] -> pair slot pslot((16l mod NH) + PB + i), component l >= 32; the
    // slots of i and i + 8 are CH + 1 apart (one pad per CH pairs)
    // (the offset is laundered: hoisted out of the sub-range loop it would be one
    // more long-lived register, spilled, with a vmcnt(0) reload)
    int po = 2 * Y::pslot(16 * (l & 31) + fu::PB) + (l >> 5);
    asm volatile("" : "+v"(po));
    float* __restrict__ pe = reinterpret_cast<float*>(P) + po;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int j = 16 * l + i;  // and j + 8
      const f2 f = bq.lp4(ef, xs[i]);
      pe[2 * i] = f.x;
      pe[2 * (i + CH + 1)] = f.y;
      if (chan_last) {
        if (j == jl) {
#pragma unroll
          for (int k = 0; k < 4; ++k) cap[k] = ef[k].x;
          have = true;
        }
        if (j + 8 == jl) {
#pragma unroll
          for (int k = 0; k < 4; ++k) cap[k] = ef[k].y;
          have = true;
        }
      }
    }
    if (have) {
      float* co = a.carry_out + ch * kWbfmCarry;
#pragma unroll
      for (int k = 0; k < 4; ++k) co[k] = cap[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      sw[k] = static_cast<double>(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(ef[k].y), 63)));
  } else {
  const double* __restrict__ lm = a.lanemats_sg;
  double ez[2][4], agg[4];
  zero_state(Bc, lm, Phi, l, xs, ez, agg);
  if (trace_r >= 0) fu::trace(a, trace_r, 10);  // debug: zero-state pass + scan done
  {  // true entering states: half A += A^{CH l} sw, half B += A^{CH l} A^NH sw
    double sB[4] = {0, 0, 0, 0};
    matvec_acc<4>(Bc.mh, sw, sB);
    matvec_acc<4>(lm + l * 16, sw, ez[0]);
    matvec_acc<4>(lm + l * 16, sB, ez[1]);
#pragma unroll
    for (int k = 0; k < 4; ++k) ef[k] = f2{static_cast<float>(ez[0][k]), static_cast<float>(ez[1][k])};
  }
  {  // pass 2 -> P[j] = (f[j], f[j + NH])
    const int jl = Lr - 1;
    float cap[4] = {0, 0, 0, 0};
    bool have = false;
    // pslot(CH l + PB + i) = pslot(CH l + PB) + i for i < CH: one base address (the
    // per-i form is not seen as linear and its eight addresses spill to scratch,
    // whose reloads wait vmcnt(0) on the prefetched tiles)
    int po = Y::pslot(CH * l + fu::PB);
    asm volatile("" : "+v"(po));  // not hoisted out of the sub-range loop (see iir16's pass 2)
    f2* __restrict__ pb = P + po;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int j = CH * l + i;
      const f2 f = bq.lp4(ef, xs[i]);
      pb[i] = f;
      if (chan_last) {
        if (j == jl) {
#pragma unroll
          for (int k = 0; k < 4; ++k) cap[k] = ef[k].x;
          have = true;
        }
        if (j + NH == jl) {
#pragma unroll
          for (int k = 0; k < 4; ++k) cap[k] = ef[k].y;
          have = true;
        }
      }
    }
    if (have) {
      float* co = a.carry_out + ch * kWbfmCarry;
#pragma unroll
      for (int k = 0; k < 4; ++k) co[k] = cap[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      sw[k] = static_cast<double>(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(ef[k].y), 63)));
  }
  }
  wave_lds_fence();
#pragma unroll
  for (int r2 = 0; r2 < 2; ++r2) {  // pairs j in [-128, 0): (history, f[j + NH])
    const int t = l + 64 * r2;
    P[Y::pslot(t)] = f2{hist[r2], P[Y::pslot(t + NH)].x};
  }
  wave_lds_fence();
#pragma unroll
  for (int r2 = 0; r2 < 2; ++r2) hist[r2] = P[Y::pslot(NH + l + 64 * r2)].y;  // f[L - 128 + t]: the next history
  if (publish_r >= 0) publish_end(a, publish_r, sw, hist, l, stride);
  if (trace_r >= 0) fu::trace(a, trace_r, 11);  // debug: IIR done
  {  // audio FIR (fir.rs:57-66), as in fu_back_range with taps in blocks of
     // KB = CH (a smaller window: this runs with two prefetched tiles live)
    constexpr int O = fu::PB - (KB - 1);  // pair index of window entry 0 at lane 0, block 0
    f2 acc[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) acc[i] = f2{0.0f, 0.0f};
#pragma unroll ORION_SEG_BACK_UNROLL
    for (int kb = 0; kb < 128 / KB; ++kb) {
      // tap k = KB kb + kk of output i reads pair e = CH l + i - k + PB
      // = CH (l - kb) + O + m, m = i + KB - 1 - kk
      const f2* __restrict__ Pl = P + (CH + 1) * (l - KB * kb / CH) + O;
      f2 w[CH + KB - 1];
#pragma unroll
      for (int m = 0; m < CH + KB - 1; ++m) w[m] = Pl[m + (O + m) / CH];
#pragma unroll
      for (int kk = 0; kk < KB; ++kk) {
        const f2 tap = splat2(Bc.a[KB * kb + kk]);
#pragma unroll
        for (int i = 0; i < CH; ++i) acc[i] = fma2(tap, w[i + KB - 1 - kk], acc[i]);
      }
    }
    float* __restrict__ y = a.y + ch * a.y_stride + A0;
    if (Lr == L && (reinterpret_cast<uintptr_t>(y) & 15) == 0) {
      float4* ya = reinterpret_cast<float4*>(y + CH * l);
      float4* yb = reinterpret_cast<float4*>(y + NH + CH * l);
#pragma unroll
      for (int i = 0; i < CH; i += 4) {
        ya[i / 4] = float4{acc[i].x, acc[i + 1].x, acc[i + 2].x, acc[i + 3].x};
        yb[i / 4] = float4{acc[i].y, acc[i + 1].y, acc[i + 2].y, acc[i + 3].y};
      }
    } else {
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int j = CH * l + i;
        if (j < Lr) y[j] = acc[i].x;
        if (j + NH < Lr) y[j + NH] = acc[i].y;
      }
    }
  }
  if (chan_last) {  // the next call's FIR history: f[n_dec - 128 .. n_dec)
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      const int t = l + 64 * r2;
      const int j = Lr - 128 + t;  // >= -128
      const float f = j < NH ? P[Y::pslot(j + fu::PB)].x : P[Y::pslot(j - NH + fu::PB)].y;
      a.carry_out[ch * kWbfmCarry + 8 + t] = f;
    }
  }
  wave_lds_fence();
  if (trace_r >= 0) fu::trace(a, trace_r, 12);  // debug: audio FIR done
}

// Publish a segment's end state and last 128 IIR outputs to its successor.
__device__ __forceinline__ void publish_end(const WbfmArgs& a, int r, const double (&sw)[4], const float (&hist)[2],
                                            int l, int stride) {
  uint32_t* slot = a.hand + static_cast<long long>(r) * stride;
  if (l < 8) {
    const int kk = l >> 1;
    const double v8 = kk == 0 ? sw[0] : kk == 1 ? sw[1] : kk == 2 ? sw[2] : sw[3];
    const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v8));
    fu::st_agent(slot + 2 + l, (l & 1) ? static_cast<uint32_t>(b >> 32) : static_cast<uint32_t>(b));
  }
  fu::st_agent(slot + 16 + l, __float_as_uint(hist[0]));
  fu::st_agent(slot + 16 + 64 + l, __float_as_uint(hist[1]));
  fu::publish(a.flags + 3LL * r, a.epoch, l);
}
}  // namespace sg

template <bool A16, bool CLAMP>
__global__ __launch_bounds__(64, 2) void k_wbfm_seg(const WbfmArgs a, const WbfmFrontConst C,
                                                    const WbfmFusedConst Bc, int spc, int S) {
  using G = fu::G;
  constexpr int TW = G::TW;
  __shared__ __attribute__((aligned(16))) f2 U[G::LDS_F2];
  __shared__ __attribute__((aligned(16))) unsigned char wreg[sg::WBytes];
  __shared__ __attribute__((aligned(16))) float Phi0[sg::L];
  __shared__ __attribute__((aligned(16))) float Gt[128];
  float* Phi = reinterpret_cast<float*>(wreg);
  f2* P = reinterpret_cast<f2*>(wreg);
  const int l = threadIdx.x & 63;
  Gt[l] = C.g[l];
  Gt[l + 64] = C.g[l + 64];
  FuRange g;
  g.r = blockIdx.x;
  g.ch = g.r / spc;
  g.wl = g.r - g.ch * spc;
  g.A = static_cast<long long>(g.wl) * S;
  g.B = min(g.A + S, a.n_dec);
  g.Lr = static_cast<int>(g.B - g.A);
  g.first = g.wl == 0;
  g.last = g.B == a.n_dec;
  const int nsub = (g.Lr + sg::L - 1) / sg::L;
  const int ntiles = nsub * sg::NS;
  const bool late = blockIdx.x >= (gridDim.x >> 1);
  fu::trace(a, g.r, 0);

  // ---- front setup (as fu_front_range) ----
  const FuPrefetch org = fu_origin(a, g);
  f2 va[G::KL][2], vb[G::KL][2];
  front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg, l, va);
  front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg + G::NEW, l, vb);
  const f2* __restrict__ tabc = a.tab + static_cast<long long>(g.ch) * kWbfmNS;
  const f2* __restrict__ xc = a.x + g.ch * a.x_stride;
  const f2* __restrict__ hc = a.hist_in + g.ch * kWbfmHist;
  const f2 cn = tabc[G::NEW];
  const int c0 = (-2 * l) & 7, c1 = (-2 * l - 1) & 7;
  const FuTile T{a, C, U, Phi0, Gt, xc, hc, tabc, g.ch, l, c0 * G::LR + (8 * Q + 2 * l + c0) / 8,
                 c1 * G::LR + (8 * Q + 2 * l + 1 + c1) / 8, f2{cn.x, -cn.y}, g.first};
  long long porg = org.porg;
  {  // halo rows of the first tile (clamped here, exact via the boundary fixup)
    const long long P0 = porg + 2 * l;
    const long long hi = (org.nl & ~1LL) - 2;
    const long long Pc = P0 < 0 ? 0 : (P0 > hi ? hi : P0);
    const f2 x0 = org.xl[Pc], x1 = org.xl[Pc + 1];
    const f4 th = *reinterpret_cast<const f4*>(tabc + 2 * l);
    U[c0 * G::LR + (2 * l + c0) / 8] = cmul_rot(x0, f2{th.x, th.y});
    U[c1 * G::LR + (2 * l + 1 + c1) / 8] = cmul_rot(x1, f2{th.z, th.w});
  }
  {  // p = -l (row c = l, i = 0), l = 1..7: used only by d[A-1]
    const long long Pm = max(porg - (l & 7), 0LL);
    const f2 xm = xc[Pm];
    const f2 tc = tabc[l & 7];
    if (!g.first && l >= 1 && l < 8) U[l * G::LR] = cmul_rot(xm, f2{tc.x, -tc.y});
  }
  f2 Sv = f2{0, 0};
  f2 carry = f2{0.0f, 0.0f}, dA = f2{0, 0};
  if (g.first) {  // d[-1]: the last decimated sample of the previous call (fm.rs:29 on reset)
    const float* ci = a.carry_in + g.ch * kWbfmCarry;
    carry = f2{ci[4], ci[5]};
  }
  double sw[4] = {0, 0, 0, 0};  // IIR state entering the next sub-range
  float hist[2] = {0, 0};       // its FIR history
  const FuPrefetch dummy{org.xl, org.nl, -8LL * Q, true};  // past the segment: an L2-resident tile

#pragma unroll 1
  for (int sub = 0, n = 0; sub < nsub; ++sub) {
    // per-lane staging phasors e^{j theta p}, p = 8Q + 2l + r + 128k: rebuilt
    // per sub-range so that they are dead (not holding 32 VGPRs) during a back
    f2 ph[G::KL][2];
    {
      const f4 tv = *reinterpret_cast<const f4*>(tabc + 8 * Q + 2 * l);
      const f2 tb0 = f2{tv.x, tv.y}, tb1 = f2{tv.z, tv.w};
#pragma unroll
      for (int k = 0; k < G::KL; ++k) {
        const f2 ek = tabc[128 * k];
        ph[k][0] = cmul(tb0, ek);
        ph[k][1] = cmul(tb1, ek);
      }
    }
    float* const dst0 = sub == 0 ? Phi0 : Phi;
#pragma unroll 1
    for (int tin = 0; tin < sg::NS; tin += 2, n += 2, porg += 2 * G::NEW) {
      // Issue priority: a SIMD's arbiter favours its oldest wave, so of the two
      // waves that share a SIMD the later-dispatched one (the upper half of the
      // grid) would run ~20% slower and leave a tail. The later wave takes the
      // higher priority for the first 10/16 of its tiles, the earlier one for
      // the rest, so both finish together.
      if (kSegPrio) {
        if ((16 * n < kSegPrioQ16 * ntiles) == late) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
      if ((n & 63) == 0)  // lane l: the common phasor of tile n + l
        Sv = phasor_q64(static_cast<uint64_t>(a.k0 + porg + 1 + static_cast<long long>(l) * G::NEW),
                        a.step[g.ch]);
      const long long jd0 = g.A + static_cast<long long>(n) * TW;
      const FuPrefetch p0 = n + 2 < ntiles ? FuPrefetch{org.xl, org.nl, porg + 2 * G::NEW, true} : dummy;
      const FuPrefetch p1 = n + 3 < ntiles ? FuPrefetch{org.xl, org.nl, porg + 3 * G::NEW, true} : dummy;
      float* dst = dst0 + TW * tin;
      fu_tile<A16, CLAMP>(T, n, porg, jd0, PhArr{ph}, va, p0, Sv, carry, dA, dst, n & 63);
      fu_tile<A16, CLAMP>(T, n + 1, porg + G::NEW, jd0 + TW, PhArr{ph}, vb, p1, Sv, carry, dA, dst + TW, (n + 1) & 63);
    }
    {  // sub-range `sub` complete: its back, with two tiles in flight
      if (sub == 0) {
        if (!(ORION_SEG_ABL & 2)) sg::zs_only(Bc, a.lanemats_sg, Phi0, Phi, l, sw, hist);
        if (nsub == 1 && !g.last) sg::publish_end(a, g.r, sw, hist, l);
      } else {
        const long long A0 = g.A + static_cast<long long>(sub) * sg::L;
        const int Lr = static_cast<int>(min(static_cast<long long>(sg::L), g.B - A0));
        const bool lastsub = sub == nsub - 1;
        if (sub <= 3) fu::trace(a, g.r, 3 + sub);  // debug: sub-range tiles done
        if (!(ORION_SEG_ABL & 1))
          sg::back(a, Bc, g.ch, A0, Lr, g.last && lastsub, Phi, P, l, sw, hist,
                   ORION_SEG_EARLY_PUB && lastsub && !g.last ? g.r : -1);
        if ((!ORION_SEG_EARLY_PUB || (ORION_SEG_ABL & 1)) && lastsub && !g.last) sg::publish_end(a, g.r, sw, hist, l);
        if (sub <= 3) fu::trace(a, g.r, 6 + sub);  // debug: its back done
      }
    }
  }
  fu::trace(a, g.r, 1);
  if (ORION_SEG_ABL & 4) {  // timing experiment: no deferred back (phi kept alive)
    if (Phi0[l] == 1234.5f && Phi[l] == 1.5f) a.y[l] = Phi0[l] + Phi[l];
    return;
  }
  // ---- deferred: sub-range 0 from the predecessor's end state ----
  if (g.first) {
    const float* __restrict__ ci = a.carry_in + g.ch * kWbfmCarry;
#pragma unroll
    for (int k = 0; k < 4; ++k) sw[k] = ci[k];
    hist[0] = ci[8 + l];
    hist[1] = ci[8 + 64 + l];
  } else {
    fu::wait_for(a.flags + 3LL * (g.r - 1), a.epoch, a.err);
    const uint32_t* ps = a.hand + static_cast<long long>(g.r - 1) * kFuSlot;
#pragma unroll
    for (int k = 0; k < 4; ++k) sw[k] = sg::uni(fu::u2d(fu::ld_agent(ps + 2 + 2 * k), fu::ld_agent(ps + 3 + 2 * k)));
    hist[0] = __uint_as_float(fu::ld_agent(ps + 16 + l));
    hist[1] = __uint_as_float(fu::ld_agent(ps + 16 + 64 + l));
  }
  fu::trace(a, g.r, 2);
  sg::back(a, Bc, g.ch, g.A, min(sg::L, g.Lr), g.last && nsub == 1, Phi0, P, l, sw, hist);
  fu::trace(a, g.r, 3);
}

// ---- segmented chain, four-group decimator ----------------------------------------
#ifndef ORION_SEG4_X
#define ORION_SEG4_X 95  // bits: 1 first phase opens the chains with a product, 2 taps-first read order (fu_tile8),
                         // 4 audio FIR in blocks of 16 taps (sg::back), 8 iir16 (16 consecutive samples per lane),
                         // 16 XCD-contiguous segment runs, 64 one tile of inputs in flight (no VGPR spills)
#endif
#ifndef ORION_SEG4_XALT
#define ORION_SEG4_XALT 95  // a second instantiation for in-process A/B (ORION_SEG4_X_LIVE=<bits>)
#endif
#ifndef ORION_SEG_PRIO_Q16_ALT
#define ORION_SEG_PRIO_Q16_ALT 9  // X & 128 (experiments): the priority hand-over point of k_wbfm_seg4, in 16ths
#endif
constexpr int kSeg4X = ORION_SEG4_X;
constexpr int kSeg4XAlt = ORION_SEG4_XALT;
// k_wbfm_seg4: k_wbfm_seg with fu_tile8's front tile. The padded image needs 2.3 KB
// more LDS, so sub-range 0's phi (kept for the deferred back) go to the segment's
// global slot (after its end-state record) instead of a third LDS buffer, and come
// back at the end (L2/MALL-resident by then).
constexpr int kSegSlot = kSeg4Slot;  // u32 words: end-state record, then sub-range 0's phi
template <bool A16, bool CLAMP, int X>
__global__ __launch_bounds__(64, 2) void k_wbfm_seg4(const WbfmArgs a, const WbfmFrontConst C,
                                                     const WbfmFusedConst Bc, int spc, int S) {
  using G = fu::G;
  constexpr int TW = G::TW;
  __shared__ __attribute__((aligned(16))) f2 U[g8::LDS_F2];
  __shared__ __attribute__((aligned(16))) unsigned char wreg[sg::WBytes];
  __shared__ __attribute__((aligned(16))) float Gt[128];
  float* Phi = reinterpret_cast<float*>(wreg);
  f2* P = reinterpret_cast<f2*>(wreg);
  const int l = threadIdx.x & 63;
  Gt[l] = C.g[l];
  Gt[l + 64] = C.g[l + 64];
  FuRange g;
  g.r = blockIdx.x;
  if constexpr ((X & 16) != 0) {
    // workgroups reach the XCDs round-robin (blockIdx % 8): give each XCD a
    // contiguous run of segments, so that a segment's predecessor (whose end
    // state it waits for) and its halo tile mostly sit on the same XCD
    const int nb = static_cast<int>(gridDim.x);
    if ((nb & 7) == 0) g.r = (blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3);
  }
  g.ch = g.r / spc;
  g.wl = g.r - g.ch * spc;
  g.A = static_cast<long long>(g.wl) * S;
  g.B = min(g.A + S, a.n_dec);
  g.Lr = static_cast<int>(g.B - g.A);
  g.first = g.wl == 0;
  g.last = g.B == a.n_dec;
  const int nsub = (g.Lr + sg::L - 1) / sg::L;
  const int ntiles = nsub * sg::NS;
  const bool late = blockIdx.x >= (gridDim.x >> 1);
  uint32_t* const myslot = a.hand + static_cast<long long>(g.r) * kSegSlot;
  fu::trace(a, g.r, 0);

  const FuPrefetch org = fu_origin(a, g);
  constexpr bool PF1 = (X & 64) != 0;  // one tile of inputs in flight instead of two (32 VGPRs)
  f2 va[G::KL][2], vb[G::KL][2];
  front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg, l, va);
  if constexpr (!PF1) front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg + G::NEW, l, vb);
  const f2* __restrict__ tabc = a.tab + static_cast<long long>(g.ch) * kWbfmNS;
  const f2* __restrict__ xc = a.x + g.ch * a.x_stride;
  const f2* __restrict__ hc = a.hist_in + g.ch * kWbfmHist;
  const f2 cn = tabc[G::NEW];
  const int c0 = (-2 * l) & 7, c1 = (-2 * l - 1) & 7;
  const FuTile T{a, C, U, Phi, Gt, xc, hc, tabc, g.ch, l, c0 * g8::LRS + g8::slot((8 * Q + 2 * l + c0) / 8),
                 c1 * g8::LRS + g8::slot((8 * Q + 2 * l + 1 + c1) / 8), f2{cn.x, -cn.y}, g.first};
  long long porg = org.porg;
  {  // halo rows of the first tile (clamped here, exact via the boundary fixup)
    const long long P0 = porg + 2 * l;
    const long long hi = (org.nl & ~1LL) - 2;
    const long long Pc = P0 < 0 ? 0 : (P0 > hi ? hi : P0);
    const f2 x0 = org.xl[Pc], x1 = org.xl[Pc + 1];
    const f4 th = *reinterpret_cast<const f4*>(tabc + 2 * l);
    U[c0 * g8::LRS + g8::slot((2 * l + c0) / 8)] = cmul_rot(x0, f2{th.x, th.y});
    U[c1 * g8::LRS + g8::slot((2 * l + 1 + c1) / 8)] = cmul_rot(x1, f2{th.z, th.w});
  }
  {  // p = -l (row c = l, entry 0), l = 1..7: used only by d[A-1]
    const long long Pm = max(porg - (l & 7), 0LL);
    const f2 xm = xc[Pm];
    const f2 tc = tabc[l & 7];
    if (!g.first && l >= 1 && l < 8) U[l * g8::LRS] = cmul_rot(xm, f2{tc.x, -tc.y});
  }
  f2 Sv = f2{0, 0};
  f2 carry = f2{0.0f, 0.0f};
  if (g.first) {
    const float* ci = a.carry_in + g.ch * kWbfmCarry;
    carry = f2{ci[4], ci[5]};
  }
  double sw[4] = {0, 0, 0, 0};
  float hist[2] = {0, 0};
  const FuPrefetch dummy{org.xl, org.nl, -8LL * Q, true};

#pragma unroll 1
  for (int sub = 0, n = 0; sub < nsub; ++sub) {
    f2 ph[G::KL][2];
    {
      const f4 tv = *reinterpret_cast<const f4*>(tabc + 8 * Q + 2 * l);
      const f2 tb0 = f2{tv.x, tv.y}, tb1 = f2{tv.z, tv.w};
#pragma unroll
      for (int k = 0; k < G::KL; ++k) {
        const f2 ek = tabc[128 * k];
        ph[k][0] = cmul(tb0, ek);
        ph[k][1] = cmul(tb1, ek);
      }
    }
    if constexpr (PF1) {
#pragma unroll 1
      for (int tin = 0; tin < sg::NS; ++tin, ++n, porg += G::NEW) {
        if (kSegPrio) {
          if ((16 * n < ((X & 128) ? ORION_SEG_PRIO_Q16_ALT : kSegPrioQ16) * ntiles) == late) __builtin_amdgcn_s_setprio(1);
          else __builtin_amdgcn_s_setprio(0);
        }
        if ((n & 63) == 0)
          Sv = phasor_q64(static_cast<uint64_t>(a.k0 + porg + 1 + static_cast<long long>(l) * G::NEW),
                          a.step[g.ch]);
        const long long jd0 = g.A + static_cast<long long>(n) * TW;
        const FuPrefetch p0 = n + 1 < ntiles ? FuPrefetch{org.xl, org.nl, porg + G::NEW, true} : dummy;
        fu_tile8<A16, CLAMP, X>(T, n, porg, jd0, ph, va, p0, Sv, carry, Phi + TW * tin, n & 63);
      }
    } else {
#pragma unroll 1
    for (int tin = 0; tin < sg::NS; tin += 2, n += 2, porg += 2 * G::NEW) {
      if (kSegPrio) {  // see k_wbfm_seg
        if ((16 * n < ((X & 128) ? ORION_SEG_PRIO_Q16_ALT : kSegPrioQ16) * ntiles) == late) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
      if ((n & 63) == 0)
        Sv = phasor_q64(static_cast<uint64_t>(a.k0 + porg + 1 + static_cast<long long>(l) * G::NEW),
                        a.step[g.ch]);
      const long long jd0 = g.A + static_cast<long long>(n) * TW;
      const FuPrefetch p0 = n + 2 < ntiles ? FuPrefetch{org.xl, org.nl, porg + 2 * G::NEW, true} : dummy;
      const FuPrefetch p1 = n + 3 < ntiles ? FuPrefetch{org.xl, org.nl, porg + 3 * G::NEW, true} : dummy;
      float* dst = Phi + TW * tin;
      fu_tile8<A16, CLAMP, X>(T, n, porg, jd0, ph, va, p0, Sv, carry, dst, n & 63);
      fu_tile8<A16, CLAMP, X>(T, n + 1, porg + G::NEW, jd0 + TW, ph, vb, p1, Sv, carry, dst + TW, (n + 1) & 63);
    }
    }  // PF1
    wave_lds_fence();
    if (sub == 0) {
      // keep sub-range 0's phi for the deferred back in the segment's global slot
      f4* gs = reinterpret_cast<f4*>(myslot + kFuSlot);
#pragma unroll
      for (int i = 0; i < sg::L / 256; ++i) gs[l + 64 * i] = *reinterpret_cast<const f4*>(Phi + 4 * (l + 64 * i));
      if constexpr ((X & 8) != 0) sg::zs_only16(Bc, Phi, Phi, l, sw, hist);
      else if (!(ORION_SEG_ABL & 2)) sg::zs_only(Bc, a.lanemats_sg, Phi, Phi, l, sw, hist);
      if (nsub == 1 && !g.last) sg::publish_end(a, g.r, sw, hist, l, kSegSlot);
    } else {
      const long long A0 = g.A + static_cast<long long>(sub) * sg::L;
      const int Lr = static_cast<int>(min(static_cast<long long>(sg::L), g.B - A0));
      const bool lastsub = sub == nsub - 1;
      if (sub <= 3) fu::trace(a, g.r, 3 + sub);
      if (!(ORION_SEG_ABL & 1))
        sg::back<(X & 4) ? 16 : ORION_SEG_BACK_KB, (X & 8) != 0>(a, Bc, g.ch, A0, Lr, g.last && lastsub, Phi, P, l, sw, hist, lastsub && !g.last ? g.r : -1,
                 kSegSlot, sub == 1 ? g.r : -1);
      else if (lastsub && !g.last)
        sg::publish_end(a, g.r, sw, hist, l, kSegSlot);
      if (sub <= 3) fu::trace(a, g.r, 6 + sub);
    }
  }
  fu::trace(a, g.r, 1);
  if (ORION_SEG_ABL & 4) return;
  // ---- deferred: sub-range 0 from the predecessor's end state ----
  {
    const f4* gs = reinterpret_cast<const f4*>(myslot + kFuSlot);
    f4 u[sg::L / 256];
#pragma unroll
    for (int i = 0; i < sg::L / 256; ++i) u[i] = __builtin_nontemporal_load(gs + l + 64 * i);
#pragma unroll
    for (int i = 0; i < sg::L / 256; ++i) *reinterpret_cast<f4*>(Phi + 4 * (l + 64 * i)) = u[i];
  }
  if (g.first) {
    const float* __restrict__ ci = a.carry_in + g.ch * kWbfmCarry;
#pragma unroll
    for (int k = 0; k < 4; ++k) sw[k] = ci[k];
    hist[0] = ci[8 + l];
    hist[1] = ci[8 + 64 + l];
  } else {
    fu::wait_for(a.flags + 3LL * (g.r - 1), a.epoch, a.err);
    const uint32_t* ps = a.hand + static_cast<long long>(g.r - 1) * kSegSlot;
#pragma unroll
    for (int k = 0; k < 4; ++k) sw[k] = sg::uni(fu::u2d(fu::ld_agent(ps + 2 + 2 * k), fu::ld_agent(ps + 3 + 2 * k)));
    hist[0] = __uint_as_float(fu::ld_agent(ps + 16 + l));
    hist[1] = __uint_as_float(fu::ld_agent(ps + 16 + 64 + l));
  }
  wave_lds_fence();
  fu::trace(a, g.r, 2);
  sg::back<(X & 4) ? 16 : ORION_SEG_BACK_KB, (X & 8) != 0>(a, Bc, g.ch, g.A, min(sg::L, g.Lr), g.last && nsub == 1, Phi, P, l, sw, hist);
  fu::trace(a, g.r, 3);
}

// ---- segmented chain, FIR-spread form ---------------------------------------------
// k_wbfm_seg2: k_wbfm_seg's one round of segments, with the back of the chain
// split so that the input stream is never held up by the audio FIR:
//   * at the end of sub-range k only its IIR runs (zero-state pass, f64 scan,
//     the reference recurrence -> the FIR pair image P, about a quarter of a
//     back), covered by the two prefetched tiles;
//   * sub-range k's audio FIR runs as 8 blocks of 16 taps, one after each front
//     tile of sub-range k+1 (P stays resident: the phi of a sub-range have an
//     LDS buffer of their own); the last sub-range's FIR runs at the end;
//   * the first sub-range of a segment that is not the channel's first needs
//     the state at the END of the previous segment. Instead of waiting for it,
//     the segment hands that sub-range's 1024 phi to its predecessor (agent-
//     scope sc1 stores + a flag, published after its first 8 tiles), and the
//     predecessor, which ends holding exactly that state and the last 128 IIR
//     outputs, runs the sub-range's IIR and FIR after its own. It reads the phi
//     long after they were published, so its wait is a formality; no wave ever
//     waits for another's end. The segment itself starts sub-range 1 from the
//     zero-state end state and zero-state last 128 outputs of sub-range 0
//     (exact to f32 when ||A^896|| is negligible: the host checks it).
#ifndef ORION_SCAN_DPP
#define ORION_SCAN_DPP 0  // 1: DPP / permlane lane shifts in the sub-range scans (measured slower: 162 vs 156 us)
#endif
namespace sg2 {
using Y = sg::Y;  // L 1024, NH 512, CH 8
constexpr int L = Y::L, NH = Y::NH, CH = Y::CH;

// LpCascade states of one sub-range (phi halves PhA = [0, NH), PhB = [NH, L))
// from its exact entering state s_in, with no
// per-lane transition matrices (those are vector loads, which would queue behind
// the in-flight tile prefetch): s_in is folded into lane 0 of half A's
// Kogge-Stone scan, half A's end state into lane 0 of half B's. xs = the lane's
// two chunks (half A, half B); ef = the state entering each (.x A, .y B), f32;
// end = the state after the sub-range (f64, wave-uniform).
__device__ __forceinline__ void scan_states(const WbfmFusedConst& Bc, const float* __restrict__ PhA,
                                            const float* __restrict__ PhB, int l, const double (&s_in)[4],
                                            f2 (&xs)[CH], f2 (&ef)[4], double (&end)[4]) {
#pragma unroll
  for (int i = 0; i < CH; i += 4) {
    const f4 u = *reinterpret_cast<const f4*>(PhA + CH * l + i);
    const f4 w = *reinterpret_cast<const f4*>(PhB + CH * l + i);
    xs[i] = f2{u.x, w.x};
    xs[i + 1] = f2{u.y, w.y};
    xs[i + 2] = f2{u.z, w.z};
    xs[i + 3] = f2{u.w, w.w};
  }
  wave_lds_fence();
  const Biquad2 bq{splat2(Bc.b0), splat2(Bc.b1), splat2(Bc.b2), splat2(Bc.a1), splat2(Bc.a2)};
  f2 s[4] = {f2{0, 0}, f2{0, 0}, f2{0, 0}, f2{0, 0}};
#pragma unroll
  for (int i = 0; i < CH; ++i) (void)bq.lp4(s, xs[i]);
  double qa[4], qb[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    qa[k] = s[k].x;
    qb[k] = s[k].y;
  }
  if (l == 0) matvec_acc<4>(Bc.pw, s_in, qa);  // pw[0] = A^CH
  if constexpr (ORION_SCAN_DPP) wave_scan_inclusive_fast<4>(qa, Bc.pw, l);
  else wave_scan_inclusive<4>(qa, Bc.pw, l);
  double sb[4];  // the state at the end of half A
#pragma unroll
  for (int k = 0; k < 4; ++k) sb[k] = sg::uni(__shfl(qa[k], 63, 64));
  if (l == 0) matvec_acc<4>(Bc.pw, sb, qb);
  if constexpr (ORION_SCAN_DPP) wave_scan_inclusive_fast<4>(qb, Bc.pw, l);
  else wave_scan_inclusive<4>(qb, Bc.pw, l);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    end[k] = sg::uni(__shfl(qb[k], 63, 64));
    const double ea = __shfl_up(qa[k], 1, 64), eb = __shfl_up(qb[k], 1, 64);
    ef[k] = f2{static_cast<float>(l == 0 ? s_in[k] : ea), static_cast<float>(l == 0 ? sb[k] : eb)};
  }
}

#ifndef ORION_IIR16
#define ORION_IIR16 0  // 1: one scan over 16-sample lane chunks (measured slower: 165 vs 157 us on C2)
#endif
// ONE Kogge-Stone over lane chunks of C16 = 16 consecutive samples of the whole
// 1024-sample sub-range instead of two chained scans over its halves (lane chunks
// of 8): 6 dependent f64 steps instead of 12 (each waits on its shuffles and on
// scalar loads of its step matrix), at the price of unpacked recurrences. Step s
// uses (A^16)^(2^s) = (A^8)^(2^(s+1)) = pw[s + 1] (s < 5) and A^512 = mh (s = 5).
constexpr int C16 = L / 64;
[[maybe_unused]] __device__ __forceinline__ void scan_states16(const WbfmFusedConst& Bc, const float* __restrict__ Ph, int l,
                                              const double (&s_in)[4], float (&xs)[C16], float (&ef)[4],
                                              double (&end)[4]) {
#pragma unroll
  for (int q = 0; q < C16 / 4; ++q) {
    const f4 u = *reinterpret_cast<const f4*>(Ph + C16 * l + 4 * q);
    xs[4 * q] = u.x;
    xs[4 * q + 1] = u.y;
    xs[4 * q + 2] = u.z;
    xs[4 * q + 3] = u.w;
  }
  wave_lds_fence();
  const RecLP4 lp{{Bc.b0, Bc.b1, Bc.b2, Bc.a1, Bc.a2}};
  float s0[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < C16; ++i) (void)lp.step(s0, xs[i]);
  double q[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) q[k] = s0[k];
  if (l == 0) matvec_acc<4>(Bc.pw + 16, s_in, q);  // A^16
#pragma unroll 1
  for (int st = 0; st < 6; ++st) {
    const int d = 1 << st;
    double o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = __shfl_up(q[k], d, 64);
    const double* m = st < 5 ? Bc.pw + 16 * (st + 1) : Bc.mh;
    if (l >= d) matvec_acc<4>(m, o, q);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    end[k] = sg::uni(__shfl(q[k], 63, 64));
    const double e = __shfl_up(q[k], 1, 64);
    ef[k] = static_cast<float>(l == 0 ? s_in[k] : e);
  }
}
// P[slot(j + PB)] = (f[j], f[j + NH]): f[j] of this lane's chunk goes to the .x
// (j < NH) or .y component of its pair.
[[maybe_unused]] __device__ __forceinline__ void put_pair(f2* P, int j, float f) {
  float* Pf = reinterpret_cast<float*>(P);
  if (j < NH) Pf[2 * Y::pslot(j + fu::PB)] = f;
  else Pf[2 * Y::pslot(j - NH + fu::PB) + 1] = f;
}

// Zero-state pass of a segment's first sub-range: its zero-state end state sw
// and zero-state last 128 outputs hist (f[L - 128 + l + 64 r]); tmp: 128 floats
// of free LDS.
// S16: the 16-sample-chunk scan (needs PhB = PhA + NH).
template <bool S16 = (ORION_IIR16 != 0)>
__device__ __forceinline__ void zs_first(const WbfmFusedConst& Bc, const float* PhA, const float* PhB, float* tmp,
                                         int l, double (&sw)[4], float (&hist)[2]) {
  if constexpr (S16) {
    constexpr int TL = 64 - fu::PB / C16;  // lanes whose chunk lies in the last 128
    const double zero[4] = {0, 0, 0, 0};
    float xs[C16], ef[4];
    scan_states16(Bc, PhA, l, zero, xs, ef, sw);
    const RecLP4 lp{{Bc.b0, Bc.b1, Bc.b2, Bc.a1, Bc.a2}};
#pragma unroll
    for (int i = 0; i < C16; ++i) {
      const float f = lp.step(ef, xs[i]);
      if (l >= TL) tmp[(l - TL) * C16 + i] = f;
    }
    wave_lds_fence();
    hist[0] = tmp[l];
    hist[1] = tmp[l + 64];
    wave_lds_fence();
    return;
  }
  constexpr int TL = 64 - fu::PB / CH;  // lanes whose half-B chunk lies in the last 128
  const double zero[4] = {0, 0, 0, 0};
  f2 xs[CH], ef[4];
  scan_states(Bc, PhA, PhB, l, zero, xs, ef, sw);
  const Biquad2 bq{splat2(Bc.b0), splat2(Bc.b1), splat2(Bc.b2), splat2(Bc.a1), splat2(Bc.a2)};
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const f2 f = bq.lp4(ef, xs[i]);
    if (l >= TL) tmp[(l - TL) * CH + i] = f.y;
  }
  wave_lds_fence();
  hist[0] = tmp[l];
  hist[1] = tmp[l + 64];
  wave_lds_fence();
}

// IIR of one sub-range [0, Lr) from its exact entering state sw and FIR history
// hist (f[-128 + l + 64 r]): the reference recurrence -> P[j] = (f[j], f[j + NH])
// for j in [-128, NH). Returns the state after f[Lr - 1] in sw and
// f[Lr - 128 + l + 64 r] in hist. chan_last: also the carried IIR state and FIR
// history of the next call.
template <bool S16 = (ORION_IIR16 != 0)>
__device__ __forceinline__ void iir(const WbfmArgs& a, const WbfmFusedConst& Bc, int ch, int Lr, bool chan_last,
                                    const float* PhA, const float* PhB, f2* P, int l, double (&sw)[4],
                                    float (&hist)[2]) {
  const int jl = Lr - 1;
  float cap[4] = {0, 0, 0, 0};
  int hl;  // the lane that computes f[jl]
  if constexpr (S16) {
    float xs[C16], ef[4];
    double end[4];
    scan_states16(Bc, PhA, l, sw, xs, ef, end);  // PhA: the whole sub-range (PhB = PhA + NH)
    const RecLP4 lp{{Bc.b0, Bc.b1, Bc.b2, Bc.a1, Bc.a2}};
    hl = jl / C16;
#pragma unroll
    for (int i = 0; i < C16; ++i) {
      const int j = C16 * l + i;
      const float f = lp.step(ef, xs[i]);
      put_pair(P, j, f);
      if (j == jl) {
#pragma unroll
        for (int k = 0; k < 4; ++k) cap[k] = ef[k];
      }
    }
  } else {
    f2 xs[CH], ef[4];
    double end[4];
    scan_states(Bc, PhA, PhB, l, sw, xs, ef, end);
    const Biquad2 bq{splat2(Bc.b0), splat2(Bc.b1), splat2(Bc.b2), splat2(Bc.a1), splat2(Bc.a2)};
    hl = jl < NH ? jl / CH : (jl - NH) / CH;
    // pslot(CH l + PB + i) = pslot(CH l + PB) + i for i < CH: one base address (the
    // per-i form is not seen as linear and its eight addresses spill to scratch,
    // whose reloads wait vmcnt(0) on the prefetched tiles)
    int po = Y::pslot(CH * l + fu::PB);
    asm volatile("" : "+v"(po));  // not hoisted out of the sub-range loop (see iir16's pass 2)
    f2* __restrict__ pb = P + po;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int j = CH * l + i;
      const f2 f = bq.lp4(ef, xs[i]);
      pb[i] = f;
      if (j == jl) {
#pragma unroll
        for (int k = 0; k < 4; ++k) cap[k] = ef[k].x;
      }
      if (j + NH == jl) {
#pragma unroll
        for (int k = 0; k < 4; ++k) cap[k] = ef[k].y;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    sw[k] = static_cast<double>(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(cap[k]), hl)));
  if (chan_last && l == 0) {
    float* co = a.carry_out + ch * kWbfmCarry;
#pragma unroll
    for (int k = 0; k < 4; ++k) co[k] = static_cast<float>(sw[k]);
  }
  wave_lds_fence();
#pragma unroll
  for (int r2 = 0; r2 < 2; ++r2) {  // pairs j in [-128, 0): (history, f[j + NH])
    const int t = l + 64 * r2;
    P[Y::pslot(t)] = f2{hist[r2], P[Y::pslot(t + NH)].x};
  }
  wave_lds_fence();
#pragma unroll
  for (int r2 = 0; r2 < 2; ++r2) {  // this sub-range's last 128 outputs: the next one's history
    const int t = l + 64 * r2;
    const int j = Lr - 128 + t;  // >= -128
    hist[r2] = j < NH ? P[Y::pslot(j + fu::PB)].x : P[Y::pslot(j - NH + fu::PB)].y;
    if (chan_last) a.carry_out[ch * kWbfmCarry + 8 + t] = hist[r2];
  }
}

// Audio FIR (fir.rs:57-66) taps 16 kb .. 16 kb + 15 of the sub-range in P, both
// halves at once (pairs): lane l owns outputs j = CH l + i and j + NH.
__device__ __forceinline__ void fir_block(const WbfmFusedConst& Bc, const f2* __restrict__ P, int l, int kb,
                                          f2 (&acc)[CH]) {
  // tap k = 16 kb + kk of output i reads pair e = CH l + i - k + PB = CH (l - 16kb/CH) + 113 + m,
  // m = i + 15 - kk; slot = e + e / CH
  const f2* __restrict__ Pl = P + (CH + 1) * (l - 16 * kb / CH) + 113;
  f2 w[CH + 15];
#pragma unroll
  for (int m = 0; m < CH + 15; ++m) w[m] = Pl[m + (113 + m) / CH];
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    const f2 tap = splat2(Bc.a[16 * kb + kk]);
#pragma unroll
    for (int i = 0; i < CH; ++i) acc[i] = fma2(tap, w[i + 15 - kk], acc[i]);
  }
}

__device__ __forceinline__ void fir_store(const WbfmArgs& a, int ch, long long A0, int Lr, int l, f2 (&acc)[CH]) {
  float* __restrict__ y = a.y + ch * a.y_stride + A0;
  if (Lr == L && (reinterpret_cast<uintptr_t>(y) & 15) == 0) {
    float4* ya = reinterpret_cast<float4*>(y + CH * l);
    float4* yb = reinterpret_cast<float4*>(y + NH + CH * l);
#pragma unroll
    for (int i = 0; i < CH; i += 4) {
      ya[i / 4] = float4{acc[i].x, acc[i + 1].x, acc[i + 2].x, acc[i + 3].x};
      yb[i / 4] = float4{acc[i].y, acc[i + 1].y, acc[i + 2].y, acc[i + 3].y};
    }
  } else {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int j = CH * l + i;
      if (j < Lr) y[j] = acc[i].x;
      if (j + NH < Lr) y[j + NH] = acc[i].y;
    }
  }
#pragma unroll
  for (int i = 0; i < CH; ++i) acc[i] = f2{0.0f, 0.0f};
}
}  // namespace sg2

template <bool A16, bool CLAMP>
__global__ __launch_bounds__(64, 2) void k_wbfm_seg2(const WbfmArgs a, const WbfmFrontConst C,
                                                     const WbfmFusedConst Bc, int spc, int S) {
  using G = fu::G;
  constexpr int TW = G::TW;
  __shared__ __attribute__((aligned(16))) f2 U[G::LDS_F2];
  __shared__ __attribute__((aligned(16))) float Phi[sg2::L];
  __shared__ __attribute__((aligned(16))) f2 P[sg2::Y::PSlots];
  __shared__ __attribute__((aligned(16))) float Gt[128];
  const int l = threadIdx.x & 63;
  Gt[l] = C.g[l];
  Gt[l + 64] = C.g[l + 64];
  FuRange g;
  g.r = blockIdx.x;
  g.ch = g.r / spc;
  g.wl = g.r - g.ch * spc;
  g.A = static_cast<long long>(g.wl) * S;
  g.B = min(g.A + S, a.n_dec);
  g.Lr = static_cast<int>(g.B - g.A);
  g.first = g.wl == 0;
  g.last = g.B == a.n_dec;
  const int nsub = (g.Lr + sg2::L - 1) / sg2::L;
  const int ntiles = nsub * sg::NS;
  const bool late = blockIdx.x >= (gridDim.x >> 1);
  fu::trace(a, g.r, 0);

  // ---- front setup (as fu_front_range) ----
  const FuPrefetch org = fu_origin(a, g);
#if ORION_SEG2_PF1
  f2 va[G::KL][2];  // one tile in flight (4 waves x 8 KB per CU already stream at 6.8 TB/s)
  f2 (&vb)[G::KL][2] = va;
  front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg, l, va);
  constexpr int PFD = 1;
#else
  f2 va[G::KL][2], vb[G::KL][2];
  front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg, l, va);
  front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg + G::NEW, l, vb);
  constexpr int PFD = 2;
#endif
  const f2* __restrict__ tabc = a.tab + static_cast<long long>(g.ch) * kWbfmNS;
  const f2* __restrict__ xc = a.x + g.ch * a.x_stride;
  const f2* __restrict__ hc = a.hist_in + g.ch * kWbfmHist;
  const f2 cn = tabc[G::NEW];
  const int c0 = (-2 * l) & 7, c1 = (-2 * l - 1) & 7;
  const FuTile T{a, C, U, Phi, Gt, xc, hc, tabc, g.ch, l, c0 * G::LR + (8 * Q + 2 * l + c0) / 8,
                 c1 * G::LR + (8 * Q + 2 * l + 1 + c1) / 8, f2{cn.x, -cn.y}, g.first};
  long long porg = org.porg;
  {  // halo rows of the first tile (clamped here, exact via the boundary fixup)
    const long long P0 = porg + 2 * l;
    const long long hi = (org.nl & ~1LL) - 2;
    const long long Pc = P0 < 0 ? 0 : (P0 > hi ? hi : P0);
    const f2 x0 = org.xl[Pc], x1 = org.xl[Pc + 1];
    const f4 th = *reinterpret_cast<const f4*>(tabc + 2 * l);
    U[c0 * G::LR + (2 * l + c0) / 8] = cmul_rot(x0, f2{th.x, th.y});
    U[c1 * G::LR + (2 * l + 1 + c1) / 8] = cmul_rot(x1, f2{th.z, th.w});
  }
  {  // p = -l (row c = l, i = 0), l = 1..7: used only by d[A-1]
    const long long Pm = max(porg - (l & 7), 0LL);
    const f2 xm = xc[Pm];
    const f2 tc = tabc[l & 7];
    if (!g.first && l >= 1 && l < 8) U[l * G::LR] = cmul_rot(xm, f2{tc.x, -tc.y});
  }
  f2 tb0, tb1;  // e^{j theta (8Q + 2l + r)}
  {
    const f4 tv = *reinterpret_cast<const f4*>(tabc + 8 * Q + 2 * l);
    tb0 = f2{tv.x, tv.y};
    tb1 = f2{tv.z, tv.w};
  }
  f2 Sv = f2{0, 0};
  f2 carry = f2{0.0f, 0.0f}, dA = f2{0, 0};
  double sw[4] = {0, 0, 0, 0};  // IIR state entering the next sub-range
  float hist[2] = {0, 0};       // its FIR history
  if (g.first) {  // the carried state of the previous call (fm.rs:29 on reset)
    const float* __restrict__ ci = a.carry_in + g.ch * kWbfmCarry;
    carry = f2{ci[4], ci[5]};
#pragma unroll
    for (int k = 0; k < 4; ++k) sw[k] = ci[k];
    hist[0] = ci[8 + l];
    hist[1] = ci[8 + 64 + l];
  }
  const FuPrefetch dummy{org.xl, org.nl, -8LL * Q, true};  // past the segment: an L2-resident tile
  f2 acc[sg2::CH];
#pragma unroll
  for (int i = 0; i < sg2::CH; ++i) acc[i] = f2{0.0f, 0.0f};
  bool pend = false;  // a sub-range's FIR spread over this sub-range's tiles
  long long pA0 = 0;
  int pLr = 0;

#pragma unroll 1
  for (int sub = 0, n = 0; sub < nsub; ++sub) {
    f2 ph[G::KL][2];  // per-lane staging phasors, rebuilt per sub-range (dead during the IIR)
    if (!ORION_SEG2_PHGEN) {  // from tb (registers) and uniform e^{j theta 128 k} (scalar loads)
#pragma unroll
      for (int k = 0; k < G::KL; ++k) {
        const f2 ek = tabc[128 * k];
        ph[k][0] = cmul(tb0, ek);
        ph[k][1] = cmul(tb1, ek);
      }
    }
#pragma unroll 1
    for (int tin = 0; tin < sg::NS; tin += 2, n += 2, porg += 2 * G::NEW) {
      if (kSegPrio) {  // see k_wbfm_seg
        if ((16 * n < kSegPrioQ16 * ntiles) == late) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
      if ((n & 63) == 0)  // lane l: the common phasor of tile n + l
        Sv = phasor_q64(static_cast<uint64_t>(a.k0 + porg + 1 + static_cast<long long>(l) * G::NEW),
                        a.step[g.ch]);
      const long long jd0 = g.A + static_cast<long long>(n) * TW;
      const FuPrefetch p0 = n + PFD < ntiles ? FuPrefetch{org.xl, org.nl, porg + PFD * G::NEW, true} : dummy;
      const FuPrefetch p1 = n + PFD + 1 < ntiles ? FuPrefetch{org.xl, org.nl, porg + (PFD + 1) * G::NEW, true} : dummy;
#if ORION_SEG2_PHGEN
      const PhGen phg = PhGen{tb0, tb1, tabc}.opaque();
#else
      const PhArr phg{ph};
#endif
      fu_tile<A16, CLAMP>(T, n, porg, jd0, phg, va, p0, Sv, carry, dA, Phi + TW * tin, n & 63);
      if (pend && !(ORION_SEG_ABL & 8)) sg2::fir_block(Bc, P, l, tin, acc);
      fu_tile<A16, CLAMP>(T, n + 1, porg + G::NEW, jd0 + TW, phg, vb, p1, Sv, carry, dA, Phi + TW * (tin + 1),
                          (n + 1) & 63);
      if (pend && !(ORION_SEG_ABL & 8)) sg2::fir_block(Bc, P, l, tin + 1, acc);
    }
    if (pend) {
      sg2::fir_store(a, g.ch, pA0, pLr, l, acc);
      pend = false;
    }
    const long long A0 = g.A + static_cast<long long>(sub) * sg2::L;
    const int Lr = static_cast<int>(min(static_cast<long long>(sg2::L), g.B - A0));
    if (sub >= 1 && sub <= 3) fu::trace(a, g.r, 3 + sub);  // debug: sub-range tiles done
    if (sub == 0 && !g.first) {
      // zero-state pass only; the phi go to the predecessor, which has the true state
      sg2::zs_first(Bc, Phi, Phi + sg2::NH, reinterpret_cast<float*>(P), l, sw, hist);
      uint32_t* slot = a.hand + static_cast<long long>(g.r) * sg2::L;
#pragma unroll
      for (int i = 0; i < sg2::L / 64; ++i) fu::st_agent(slot + l + 64 * i, __float_as_uint(Phi[l + 64 * i]));
      fu::publish(a.flags + 3LL * g.r, a.epoch, l);
    } else if (!(ORION_SEG_ABL & 1)) {
      sg2::iir(a, Bc, g.ch, Lr, g.last && sub == nsub - 1, Phi, Phi + sg2::NH, P, l, sw, hist);
      if (sub <= 3) fu::trace(a, g.r, 6 + sub);  // debug: its IIR done
      pend = true;
      pA0 = A0;
      pLr = Lr;
    }
  }
  fu::trace(a, g.r, 1);
  // End of the segment: the successor's first sub-range needs this segment's end
  // state (sw, hist: known now). Its IIR runs first, its FIR pair image in the
  // front image U (dead after the last tile), and then the two audio FIRs (this
  // segment's last sub-range and the successor's) run interleaved: two
  // independent accumulator sets, twice the FMA chains per LDS window.
  const bool succ = !g.last && !(ORION_SEG_ABL & 4);
  f2* const P2 = U;
  long long As = 0;
  int Lrs = 0;
  if (succ) {  // the successor segment's first sub-range
    As = g.B;
    const long long Bs = min(As + S, a.n_dec);
    Lrs = static_cast<int>(min(static_cast<long long>(sg2::L), Bs - As));
    const bool s_last = Bs == a.n_dec && Bs - As <= sg2::L;
    fu::wait_for(a.flags + 3LL * (g.r + 1), a.epoch, a.err);
    fu::trace(a, g.r, 2);
    const uint32_t* slot = a.hand + static_cast<long long>(g.r + 1) * sg2::L;
#pragma unroll
    for (int i = 0; i < sg2::L / 64; ++i) Phi[l + 64 * i] = __uint_as_float(fu::ld_agent(slot + l + 64 * i));
    wave_lds_fence();
    sg2::iir(a, Bc, g.ch, Lrs, s_last, Phi, Phi + sg2::NH, P2, l, sw, hist);
  }
  if (pend || succ) {
    f2 acc2[sg2::CH];
#pragma unroll
    for (int i = 0; i < sg2::CH; ++i) acc2[i] = f2{0.0f, 0.0f};
#pragma unroll 1
    for (int kb = 0; kb < 8; ++kb) {
      if (pend) sg2::fir_block(Bc, P, l, kb, acc);
      if (succ) sg2::fir_block(Bc, P2, l, kb, acc2);
    }
    if (pend) sg2::fir_store(a, g.ch, pA0, pLr, l, acc);
    if (succ) sg2::fir_store(a, g.ch, As, Lrs, l, acc2);
  }
  fu::trace(a, g.r, 3);
}

// ---- segmented chain, three waves per SIMD ------------------------------------------
// k_wbfm_seg3: k_wbfm_seg2's one round of segments and first-sub-range hand-off,
// sized for THREE waves per SIMD (<= 168 VGPRs, <= 13.6 KB of LDS per wave): the
// wave count, not the instruction count, bounds this chain (2048 -> 1792 -> 1536
// segments: 160 -> 175 -> 200 us), so a third wave per SIMD is worth a leaner
// wave:
//   * the back of a sub-range (IIR, then the whole audio FIR) runs as one burst
//     right after its last tile, with two tiles of inputs in flight, and its FIR
//     pair image P aliases the front image U: the 17-column halo the next tile
//     needs is carried across the burst in registers (already times e^{-j theta
//     NEW}, as fu_tile's copy would make it);
//   * staging phasors are formed per tile (PhGen), not held (32 VGPRs);
//   * no LDS tap copy: the one-off d[A-1] sum reads the taps from global memory.
#ifndef ORION_SEG3_ABL
#define ORION_SEG3_ABL 0  // register/timing experiments: 1 no sub-range bursts, 2 no successor sub-range
#endif
namespace sg3 {
using sg2::CH;
using sg2::L;
using sg2::NH;
constexpr int kHaloLanes = 72;  // f4 pairs of the halo: 8 rows x 9

// The halo of the next tile, e^{-j theta NEW} applied (fu_tile's copy), saved
// before P overwrites U and written back to the row heads after the burst.
struct Halo {
  f4 h[2];
  __device__ __forceinline__ void save(const f2* U, f2 corr, int l) {
    using G = fu::G;
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      const int e = l + 64 * r2;
      if (e < kHaloLanes) {
        const int c = e / 9, hh = e - 9 * c;
        const f4 w = *reinterpret_cast<const f4*>(U + c * G::LR + G::TW + 2 * hh);
        const f2 y0 = cmul(f2{w.x, w.y}, corr), y1 = cmul(f2{w.z, w.w}, corr);
        h[r2] = f4{y0.x, y0.y, y1.x, y1.y};
      }
    }
  }
  __device__ __forceinline__ void restore(f2* U, int l) const {
    using G = fu::G;
#pragma unroll
    for (int r2 = 0; r2 < 2; ++r2) {
      const int e = l + 64 * r2;
      if (e < kHaloLanes) {
        const int c = e / 9, hh = e - 9 * c;
        *reinterpret_cast<f4*>(U + c * G::LR + 2 * hh) = h[r2];
      }
    }
  }
};

// IIR + whole audio FIR of one sub-range, P in U (the caller saved the halo).
__device__ __forceinline__ void burst(const WbfmArgs& a, const WbfmFusedConst& Bc, int ch, long long A0, int Lr,
                                      bool chan_last, const float* Phi, f2* P, int l, double (&sw)[4],
                                      float (&hist)[2]) {
  if (!(ORION_SEG3_ABL & 4)) sg2::iir(a, Bc, ch, Lr, chan_last, Phi, Phi + NH, P, l, sw, hist);
  wave_lds_fence();
  if (ORION_SEG3_ABL & 8) return;
  // audio FIR (fir.rs:57-66) in blocks of KB = 8 taps (a 15-pair window: this runs
  // with two prefetched tiles live); lane l owns outputs j = CH l + i and j + NH
  constexpr int KB = 8;
  constexpr int O = fu::PB - (KB - 1);  // pair index of window entry 0 at lane 0, block 0
  f2 acc[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) acc[i] = f2{0.0f, 0.0f};
#pragma unroll 1
  for (int kb = 0; kb < 128 / KB; ++kb) {
    // tap k = KB kb + kk of output i reads pair e = CH l + i - k + PB = CH (l - kb) + O + m,
    // m = i + KB - 1 - kk; slot = e + e / CH
    const f2* __restrict__ Pl = P + (CH + 1) * (l - KB * kb / CH) + O;
    f2 w[CH + KB - 1];
#pragma unroll
    for (int m = 0; m < CH + KB - 1; ++m) w[m] = Pl[m + (O + m) / CH];
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      const f2 tap = splat2(Bc.a[KB * kb + kk]);
#pragma unroll
      for (int i = 0; i < CH; ++i) acc[i] = fma2(tap, w[i + KB - 1 - kk], acc[i]);
    }
  }
  sg2::fir_store(a, ch, A0, Lr, l, acc);
  wave_lds_fence();
}
}  // namespace sg3

static_assert(fu::G::LDS_F2 * 8 + sg2::L * 4 <= 163840 / 12, "three waves per SIMD: LDS per wave");
static_assert(sg2::Y::PSlots <= fu::G::LDS_F2, "the FIR pair image fits the front image");

template <bool A16, bool CLAMP>
__global__ __launch_bounds__(64, 3) void k_wbfm_seg3(const WbfmArgs a, const WbfmFrontConst C,
                                                     const WbfmFusedConst Bc, int spc, int S) {
  using G = fu::G;
  constexpr int TW = G::TW;
  __shared__ __attribute__((aligned(16))) f2 U[G::LDS_F2];
  __shared__ __attribute__((aligned(16))) float Phi[sg2::L];
  f2* const P = U;
  const int l = threadIdx.x & 63;
  FuRange g;
  g.r = blockIdx.x;
  g.ch = g.r / spc;
  g.wl = g.r - g.ch * spc;
  g.A = static_cast<long long>(g.wl) * S;
  g.B = min(g.A + S, a.n_dec);
  g.Lr = static_cast<int>(g.B - g.A);
  g.first = g.wl == 0;
  g.last = g.B == a.n_dec;
  const int nsub = (g.Lr + sg2::L - 1) / sg2::L;
  const int ntiles = nsub * sg::NS;
  fu::trace(a, g.r, 0);

  const FuPrefetch org = fu_origin(a, g);
  f2 va[G::KL][2];  // ONE tile in flight: 12 waves per CU keep 96 KB of loads in flight
  front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg, l, va);
  const f2* __restrict__ tabc = a.tab + static_cast<long long>(g.ch) * kWbfmNS;
  const f2* __restrict__ xc = a.x + g.ch * a.x_stride;
  const f2* __restrict__ hc = a.hist_in + g.ch * kWbfmHist;
  const f2 cn = tabc[G::NEW];
  const int c0 = (-2 * l) & 7, c1 = (-2 * l - 1) & 7;
  const FuTile T{a, C, U, Phi, C.g, xc, hc, tabc, g.ch, l, c0 * G::LR + (8 * Q + 2 * l + c0) / 8,
                 c1 * G::LR + (8 * Q + 2 * l + 1 + c1) / 8, f2{cn.x, -cn.y}, g.first};
  long long porg = org.porg;
  {  // halo rows of the first tile (clamped here, exact via the boundary fixup)
    const long long P0 = porg + 2 * l;
    const long long hi = (org.nl & ~1LL) - 2;
    const long long Pc = P0 < 0 ? 0 : (P0 > hi ? hi : P0);
    const f2 x0 = org.xl[Pc], x1 = org.xl[Pc + 1];
    const f4 th = *reinterpret_cast<const f4*>(tabc + 2 * l);
    U[c0 * G::LR + (2 * l + c0) / 8] = cmul_rot(x0, f2{th.x, th.y});
    U[c1 * G::LR + (2 * l + 1 + c1) / 8] = cmul_rot(x1, f2{th.z, th.w});
  }
  {  // p = -l (row c = l, i = 0), l = 1..7: used only by d[A-1]
    const long long Pm = max(porg - (l & 7), 0LL);
    const f2 xm = xc[Pm];
    const f2 tc = tabc[l & 7];
    if (!g.first && l >= 1 && l < 8) U[l * G::LR] = cmul_rot(xm, f2{tc.x, -tc.y});
  }
  f2 tb0, tb1;  // e^{j theta (8Q + 2l + r)}
  {
    const f4 tv = *reinterpret_cast<const f4*>(tabc + 8 * Q + 2 * l);
    tb0 = f2{tv.x, tv.y};
    tb1 = f2{tv.z, tv.w};
  }
  f2 Sv = f2{0, 0};
  f2 carry = f2{0.0f, 0.0f}, dA = f2{0, 0};
  double sw[4] = {0, 0, 0, 0};  // IIR state entering the next sub-range
  float hist[2] = {0, 0};       // its FIR history
  if (g.first) {  // the carried state of the previous call (fm.rs:29 on reset)
    const float* __restrict__ ci = a.carry_in + g.ch * kWbfmCarry;
    carry = f2{ci[4], ci[5]};
#pragma unroll
    for (int k = 0; k < 4; ++k) sw[k] = ci[k];
    hist[0] = ci[8 + l];
    hist[1] = ci[8 + 64 + l];
  }
  const FuPrefetch dummy{org.xl, org.nl, -8LL * Q, true};  // past the segment: an L2-resident tile
  bool halo_ok = true;  // U's head halo is in place (false: fu_tile copies it)
  sg3::Halo halo;

#pragma unroll 1
  for (int sub = 0, n = 0; sub < nsub; ++sub) {
#pragma unroll 1
    for (int tin = 0; tin < sg::NS; tin += 2, n += 2, porg += 2 * G::NEW) {
      if ((n & 63) == 0)  // lane l: the common phasor of tile n + l
        Sv = phasor_q64(static_cast<uint64_t>(a.k0 + porg + 1 + static_cast<long long>(l) * G::NEW),
                        a.step[g.ch]);
      const long long jd0 = g.A + static_cast<long long>(n) * TW;
      const FuPrefetch p0 = n + 1 < ntiles ? FuPrefetch{org.xl, org.nl, porg + G::NEW, true} : dummy;
      const FuPrefetch p1 = n + 2 < ntiles ? FuPrefetch{org.xl, org.nl, porg + 2 * G::NEW, true} : dummy;
      const PhGen phg = PhGen{tb0, tb1, tabc}.opaque();
      fu_tile<A16, CLAMP>(T, n, porg, jd0, phg, va, p0, Sv, carry, dA, Phi + TW * tin, n & 63, halo_ok);
      fu_tile<A16, CLAMP>(T, n + 1, porg + G::NEW, jd0 + TW, phg, va, p1, Sv, carry, dA, Phi + TW * (tin + 1),
                          (n + 1) & 63);
      halo_ok = true;
    }
    const long long A0 = g.A + static_cast<long long>(sub) * sg2::L;
    const int Lr = static_cast<int>(min(static_cast<long long>(sg2::L), g.B - A0));
    if (sub == 0 && !g.first) {
      // zero-state pass only; the phi go to the predecessor, which has the true state
      // (scratch: U's row-0 head, which the next tile's halo copy and staging rewrite)
      sg2::zs_first(Bc, Phi, Phi + sg2::NH, reinterpret_cast<float*>(U), l, sw, hist);
      uint32_t* slot = a.hand + static_cast<long long>(g.r) * sg2::L;
#pragma unroll
      for (int i = 0; i < sg2::L / 64; ++i) fu::st_agent(slot + l + 64 * i, __float_as_uint(Phi[l + 64 * i]));
      fu::publish(a.flags + 3LL * g.r, a.epoch, l);
    } else {
      wave_lds_fence();
      halo.save(U, T.corr, l);
      wave_lds_fence();
      if (!(ORION_SEG3_ABL & 1)) sg3::burst(a, Bc, g.ch, A0, Lr, g.last && sub == nsub - 1, Phi, P, l, sw, hist);
      halo.restore(U, l);
      halo_ok = false;
    }
  }
  fu::trace(a, g.r, 1);
  if (!g.last && !(ORION_SEG3_ABL & 2)) {  // the successor segment's first sub-range
    const long long As = g.B, Bs = min(As + S, a.n_dec);
    const int Lrs = static_cast<int>(min(static_cast<long long>(sg2::L), Bs - As));
    const bool s_last = Bs == a.n_dec && Bs - As <= sg2::L;
    fu::wait_for(a.flags + 3LL * (g.r + 1), a.epoch, a.err);
    fu::trace(a, g.r, 2);
    const uint32_t* slot = a.hand + static_cast<long long>(g.r + 1) * sg2::L;
#pragma unroll
    for (int i = 0; i < sg2::L / 64; ++i) Phi[l + 64 * i] = __uint_as_float(fu::ld_agent(slot + l + 64 * i));
    wave_lds_fence();
    sg3::burst(a, Bc, g.ch, As, Lrs, s_last, Phi, P, l, sw, hist);
  }
  fu::trace(a, g.r, 3);
}

// ---- k_wbfm_ws: wave-specialised segments ------------------------------------
// One 12-wave workgroup per CU (3 waves per SIMD, <= 168 VGPRs each): waves 0-7
// stream, each the front tiles of its own segment with two tiles of inputs in
// flight (as many streaming waves per SIMD as k_wbfm_seg2, but none of them
// stops for IIR or FIR work while it streams, which would let its prefetch run
// dry); waves 8-11 each run the back (IIR, audio FIR) of two streams' sub-ranges
// (streams w - 8 and w - 4, alternating), all but the last one of each.
// Phi travel through a per-stream ring of three 512-float halves in LDS: the
// front writes sub-range s into halves 2s, 2s+1 (mod 3) and bumps `prod`; the
// back reads both halves into registers and bumps `cons`; the front re-uses a
// half only once the sub-range that held it has been consumed, which leaves the
// back a sub-range and a half of slack. A wave's DS operations complete in
// order, so the phi land before the counter that announces them.
// Segment ends: when a stream's tiles are done, its own wave runs the last
// sub-range (the back parks the IIR state and FIR history in the free ring
// half, then bumps `done`) and the successor segment's first sub-range, handed
// over as in k_wbfm_seg2 (a segment's first sub-range goes to its predecessor,
// which has the true state). Eight streaming waves share that tail work instead
// of four back waves running four sub-ranges each.
#ifndef ORION_WS_ABL
#define ORION_WS_ABL 0  // timing experiments only: 1 back waves only release the ring, 2 fronts never wait
#endif
#ifndef ORION_WS_PRIO
#define ORION_WS_PRIO 1  // 1: streaming waves take s_setprio 1; 2: back waves do; 0: neither
#endif
namespace ws {
#ifndef ORION_WS_NFR
#define ORION_WS_NFR 8  // streaming waves per workgroup: 8 (3 waves per SIMD) or 4 (2 per SIMD)
#endif
constexpr int NFR = ORION_WS_NFR;                 // streaming waves per workgroup
constexpr int NBK = 4;                            // back waves
constexpr int SPB = NFR / NBK;                    // streams per back wave (1 or 2)
static_assert(SPB == 1 || SPB == 2, "geometry");
#ifndef ORION_WS_D
#define ORION_WS_D 2  // tiles in flight per streaming wave (2, or 4 with 4 streaming waves)
#endif
constexpr int D = ORION_WS_D;
static_assert(D == 2 || D == 4, "prefetch depth divides the 8 tiles of a sub-range");
constexpr int HALF = sg2::NH;                     // ring granule (512 phi)
constexpr int UF = (fu::G::LDS_F2 + 1) & ~1;      // per-stream front image (16-B aligned)
constexpr int PF = (sg2::Y::PSlots + 1) & ~1;     // per-back-wave FIR pair image
static_assert(PF <= UF, "a stream's FIR pair image fits its front image");
constexpr int kThreads = 64 * (NFR + NBK);
__device__ __forceinline__ int lds_ld(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// bounded: a wait that never ends sets *err and lets the wave finish
__device__ __forceinline__ void wait_ge(const int* p, int v, int* err) {
  for (int it = 0; lds_ld(p) < v; ++it) {
    if (it == (1 << 24)) {
      __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
}

// One sub-range's back from phi halves PhA, PhB: a segment's first sub-range
// (not the channel's) is the zero-state pass and the hand-off to the
// predecessor; any other runs the IIR, releases the phi (*rel = sub + 1, when
// rel) and the audio FIR.
__device__ __forceinline__ void job(const WbfmArgs& a, const WbfmFusedConst& Bc, const FuRange& g, int sub,
                                    bool chan_last, const float* PhA, const float* PhB, f2* P, int l,
                                    double (&sw)[4], float (&hist)[2], int* rel) {
  const long long A0 = g.A + static_cast<long long>(sub) * sg2::L;
  const int Lr = static_cast<int>(min(static_cast<long long>(sg2::L), g.B - A0));
  if (sub == 0 && !g.first) {
    sg2::zs_first<false>(Bc, PhA, PhB, reinterpret_cast<float*>(P), l, sw, hist);
    uint32_t* slot = a.hand + static_cast<long long>(g.r) * sg2::L;
#pragma unroll
    for (int i = 0; i < sg2::L / 64; ++i)
      fu::st_agent(slot + l + 64 * i, __float_as_uint((i < 8 ? PhA : PhB - sg2::NH)[l + 64 * i]));
    wave_lds_fence();
    if (rel && l == 0) lds_st(rel, sub + 1);
    fu::publish(a.flags + 3LL * g.r, a.epoch, l);
  } else {
    sg2::iir<false>(a, Bc, g.ch, Lr, chan_last, PhA, PhB, P, l, sw, hist);
    if (rel && l == 0) lds_st(rel, sub + 1);  // iir read the phi first (scan_states)
    f2 acc[sg2::CH];
#pragma unroll
    for (int i = 0; i < sg2::CH; ++i) acc[i] = f2{0.0f, 0.0f};
#pragma unroll 1
    for (int kb = 0; kb < 8; ++kb) sg2::fir_block(Bc, P, l, kb, acc);
    sg2::fir_store(a, g.ch, A0, Lr, l, acc);
  }
}
}  // namespace ws

template <bool A16, bool CLAMP>
__global__ __launch_bounds__(ws::kThreads, 1) void k_wbfm_ws(const WbfmArgs a, const WbfmFrontConst C,
                                                            const WbfmFusedConst Bk, int spc, int S, int nseg) {
  using G = fu::G;
  constexpr int TW = G::TW;
  __shared__ __attribute__((aligned(16))) f2 Us[ws::NFR * ws::UF];
  __shared__ __attribute__((aligned(16))) float Ring[ws::NFR][3][ws::HALF];
  __shared__ __attribute__((aligned(16))) f2 Ps[ws::NBK * ws::PF];
  __shared__ __attribute__((aligned(16))) float Gt[128];        // decimator taps (phase-major)
  __shared__ __attribute__((aligned(16))) f2 SvL[ws::NFR][64];  // common phasors of 64 tiles
  __shared__ __attribute__((aligned(16))) f4 TbL[ws::NFR][64];  // lane base phasors
  __shared__ double SwL[ws::NBK][8];                            // back: parked IIR states
  __shared__ int Sync[ws::NFR][3];  // [prod, cons, done] per stream
  // the back's constants in LDS (read through a kernel-argument reference in two
  // roles, the compiler copied them to scratch)
  __shared__ __attribute__((aligned(16))) WbfmFusedConst Bc;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x < 3 * ws::NFR) Sync[threadIdx.x / 3][threadIdx.x % 3] = 0;
  if (threadIdx.x < 128) Gt[threadIdx.x] = C.g[threadIdx.x];
  static_assert(sizeof(WbfmFusedConst) % 4 == 0 && sizeof(WbfmFusedConst) / 4 <= ws::kThreads, "one word per lane");
  if (threadIdx.x < sizeof(WbfmFusedConst) / 4)
    reinterpret_cast<uint32_t*>(&Bc)[threadIdx.x] = reinterpret_cast<const uint32_t*>(&Bk)[threadIdx.x];
  __syncthreads();  // the only barrier: before any load is in flight
  auto seg = [&](int f) {
    FuRange g;
    g.r = blockIdx.x * ws::NFR + f;
    g.ch = g.r / spc;
    g.wl = g.r - g.ch * spc;
    g.A = static_cast<long long>(g.wl) * S;
    g.B = min(g.A + S, a.n_dec);
    g.Lr = static_cast<int>(g.B - g.A);
    g.first = g.wl == 0;
    g.last = g.B == a.n_dec;
    return g;
  };

  if (w < ws::NFR) {  // ---- streaming wave ----
    const int f = w;
    if (blockIdx.x * ws::NFR + f >= nseg) return;
    if (ORION_WS_PRIO == 1) __builtin_amdgcn_s_setprio(1);
    const FuRange g = seg(f);
    fu::trace(a, g.r, 0);
    int* prod = &Sync[f][0];
    const int* cons = &Sync[f][1];
    f2* U = Us + f * ws::UF;
    const int nsub = (g.Lr + sg2::L - 1) / sg2::L;
    const int ntiles = nsub * sg::NS;
    const FuPrefetch org = fu_origin(a, g);
    f2 v[ws::D][G::KL][2];
#pragma unroll
    for (int j = 0; j < ws::D; ++j) front2_load<2, A16, CLAMP>(org.xl, org.nl, org.porg + j * G::NEW, l, v[j]);
    const f2* __restrict__ tabc = a.tab + static_cast<long long>(g.ch) * kWbfmNS;
    const f2* __restrict__ xc = a.x + g.ch * a.x_stride;
    const f2* __restrict__ hc = a.hist_in + g.ch * kWbfmHist;
    const f2 cn = tabc[G::NEW];
    const int c0 = (-2 * l) & 7, c1 = (-2 * l - 1) & 7;
    // the tile's scatter slots, re-derived per tile from an opaque lane index
    // (registers are the streaming wave's limit: a hoisted copy would spill)
    auto tile = [&]() {
      int lo = l;
      asm volatile("" : "+v"(lo));
      const int d0 = (-2 * lo) & 7, d1 = (-2 * lo - 1) & 7;
      return FuTile{a, C, U, Ring[f][0], Gt, xc, hc, tabc, g.ch, lo, d0 * G::LR + (8 * Q + 2 * lo + d0) / 8,
                    d1 * G::LR + (8 * Q + 2 * lo + 1 + d1) / 8, f2{cn.x, -cn.y}, g.first};
    };
    long long porg = org.porg;
    {  // halo rows of the first tile (clamped here, exact via the boundary fixup)
      const long long P0 = porg + 2 * l;
      const long long hi = (org.nl & ~1LL) - 2;
      const long long Pc = P0 < 0 ? 0 : (P0 > hi ? hi : P0);
      const f2 x0 = org.xl[Pc], x1 = org.xl[Pc + 1];
      const f4 th = *reinterpret_cast<const f4*>(tabc + 2 * l);
      U[c0 * G::LR + (2 * l + c0) / 8] = cmul_rot(x0, f2{th.x, th.y});
      U[c1 * G::LR + (2 * l + 1 + c1) / 8] = cmul_rot(x1, f2{th.z, th.w});
    }
    {  // p = -l (row c = l, i = 0), l = 1..7: used only by d[A-1]
      const long long Pm = max(porg - (l & 7), 0LL);
      const f2 xm = xc[Pm];
      const f2 tc = tabc[l & 7];
      if (!g.first && l >= 1 && l < 8) U[l * G::LR] = cmul_rot(xm, f2{tc.x, -tc.y});
    }
    // staging phasors formed per tile from the lane's two base phasors, parked
    // in LDS (registers are the streaming wave's limit)
    TbL[f][l] = *reinterpret_cast<const f4*>(tabc + 8 * Q + 2 * l);
    auto ph = [&]() {
      const f4 tv = TbL[f][l];
      return PhGen{f2{tv.x, tv.y}, f2{tv.z, tv.w}, tabc};
    };
    f2 carry = f2{0.0f, 0.0f}, dA = f2{0, 0};
    if (g.first) {  // d[-1]: the previous call's last decimated sample (fm.rs:29 on reset)
      const float* __restrict__ ci = a.carry_in + g.ch * kWbfmCarry;
      carry = f2{ci[4], ci[5]};
    }
    const FuPrefetch dummy{org.xl, org.nl, -8LL * Q, true};  // past the segment: an L2-resident tile
#pragma unroll 1
    for (int n = 0; n < ntiles; n += ws::D, porg += ws::D * G::NEW) {
      if ((n & 63) == 0) {  // lane l: the common phasor of tile n + l (kept in LDS)
        SvL[f][l] = phasor_q64(static_cast<uint64_t>(a.k0 + porg + 1 + static_cast<long long>(l) * G::NEW),
                               a.step[g.ch]);
        wave_lds_fence();
      }
#pragma unroll
      for (int j = 0; j < ws::D; ++j) {
        const int nj = n + j, sub = nj >> 3, tin = nj & 7;
        // ring half 2 sub + (tin >= 4) re-uses the half of sub-range sub - 2 + (tin >= 4)
        if (!(ORION_WS_ABL & 2) && tin == 0 && sub >= 2) ws::wait_ge(cons, sub - 1, a.err);
        if (!(ORION_WS_ABL & 2) && tin == 4 && sub >= 1) ws::wait_ge(cons, sub, a.err);
        float* phj = Ring[f][(2 * sub + (tin >> 2)) % 3] + TW * (tin & 3);
        const long long pj = porg + j * G::NEW;
        const FuPrefetch pf = nj + ws::D < ntiles ? FuPrefetch{org.xl, org.nl, pj + ws::D * G::NEW, true} : dummy;
        fu_tile<A16, CLAMP>(tile(), nj, pj, g.A + static_cast<long long>(nj) * TW, ph(), v[j], pf,
                            SvL[f][nj & 63], carry, dA, phj, 0);
        if (tin == 7) {
          wave_lds_fence();
          if (l == 0) ws::lds_st(prod, sub + 1);
        }
      }
    }
    fu::trace(a, g.r, 1);
    if (ORION_WS_ABL & 1) return;
    // ---- the segment's last sub-range, then the successor's first ----
    // (geometry re-derived from an opaque stream index: nothing stays live
    // across the tile loop for this part)
    int fo = __builtin_amdgcn_readfirstlane(f);
    asm volatile("" : "+s"(fo));
    const FuRange gt = seg(fo);
    const int s = (gt.Lr + sg2::L - 1) / sg2::L - 1;
    f2* P = reinterpret_cast<f2*>(Us + fo * ws::UF);  // the front image is free now
    double sw[4] = {0, 0, 0, 0};
    float hist[2] = {0, 0};
    if (s > 0) {  // the back parked the state after sub-range s - 1
      ws::wait_ge(&Sync[fo][2], 1, a.err);
      const float* park = Ring[fo][(2 * s + 2) % 3];
#pragma unroll
      for (int k = 0; k < 4; ++k) sw[k] = sg::uni(reinterpret_cast<const double*>(park + 128)[k]);
      hist[0] = park[l];
      hist[1] = park[64 + l];
    } else if (gt.first) {
      const float* __restrict__ ci = a.carry_in + gt.ch * kWbfmCarry;
#pragma unroll
      for (int k = 0; k < 4; ++k) sw[k] = ci[k];
      hist[0] = ci[8 + l];
      hist[1] = ci[8 + 64 + l];
    }
    {
      const float* PhA = Ring[fo][(2 * s) % 3];
      const float* PhB = Ring[fo][(2 * s + 1) % 3];
      const long long A0 = gt.A + static_cast<long long>(s) * sg2::L;
      const int Lr = static_cast<int>(min(static_cast<long long>(sg2::L), gt.B - A0));
      if (s == 0 && !gt.first) {
        sg2::zs_first<false>(Bc, PhA, PhB, reinterpret_cast<float*>(P), l, sw, hist);
        uint32_t* slot = a.hand + static_cast<long long>(gt.r) * sg2::L;
#pragma unroll
        for (int i = 0; i < sg2::L / 64; ++i)
          fu::st_agent(slot + l + 64 * i, __float_as_uint((i < 8 ? PhA : PhB - sg2::NH)[l + 64 * i]));
        fu::publish(a.flags + 3LL * gt.r, a.epoch, l);
      } else {
        sg2::iir<false>(a, Bc, gt.ch, Lr, gt.last, PhA, PhB, P, l, sw, hist);
        f2 acc[sg2::CH];
#pragma unroll
        for (int i = 0; i < sg2::CH; ++i) acc[i] = f2{0.0f, 0.0f};
#pragma unroll 1
        for (int kb = 0; kb < 8; ++kb) sg2::fir_block(Bc, P, l, kb, acc);
        sg2::fir_store(a, gt.ch, A0, Lr, l, acc);
      }
    }
    fu::trace(a, gt.r, 2);
    if (!gt.last) {
      const long long As = gt.B, Bs = min(As + S, a.n_dec);
      const int Lrs = static_cast<int>(min(static_cast<long long>(sg2::L), Bs - As));
      const bool s_last = Bs == a.n_dec && Bs - As <= sg2::L;
      float* Ph = Ring[fo][0];  // halves 0, 1: the ring is free
      fu::wait_for(a.flags + 3LL * (gt.r + 1), a.epoch, a.err);
      const uint32_t* slot = a.hand + static_cast<long long>(gt.r + 1) * sg2::L;
      wave_lds_fence();  // the last job's LDS reads are done before the ring is overwritten
#pragma unroll
      for (int i = 0; i < sg2::L / 64; ++i) Ph[l + 64 * i] = __uint_as_float(fu::ld_agent(slot + l + 64 * i));
      wave_lds_fence();
      sg2::iir(a, Bc, gt.ch, Lrs, s_last, Ph, Ph + sg2::NH, P, l, sw, hist);
      f2 acc[sg2::CH];
#pragma unroll
      for (int i = 0; i < sg2::CH; ++i) acc[i] = f2{0.0f, 0.0f};
#pragma unroll 1
      for (int kb = 0; kb < 8; ++kb) sg2::fir_block(Bc, P, l, kb, acc);
      sg2::fir_store(a, gt.ch, As, Lrs, l, acc);
    }
    fu::trace(a, g.r, 3);
    return;
  }

  // ---- back wave: sub-ranges 0 .. nsub-2 of streams b and b + NBK, alternating ----
  const int b = w - ws::NFR;
  if (ORION_WS_PRIO == 2) __builtin_amdgcn_s_setprio(1);
  f2* P = Ps + b * ws::PF;
  auto nsub_of = [&](int q) {
    const int f = b + ws::NBK * q;
    return blockIdx.x * ws::NFR + f < nseg ? (seg(f).Lr + sg2::L - 1) / sg2::L : 0;
  };
  const int nsub0 = nsub_of(0), nsub1 = ws::SPB > 1 ? nsub_of(1) : 0;
  if (nsub0 == 0) return;  // stream b + NBK exists only if stream b does
  // per stream: the IIR state entering its next sub-range (parked in LDS: SGPRs
  // are short here) and its FIR history (registers)
  double* swL = SwL[b];
  float hi0[2] = {0, 0}, hi1[2] = {0, 0};
#pragma unroll
  for (int q = 0; q < ws::SPB; ++q) {
    const FuRange g = seg(b + ws::NBK * q);
    const bool carried = (q ? nsub1 : nsub0) > 0 && g.first;
    const float* __restrict__ ci = a.carry_in + g.ch * kWbfmCarry;
    if (l < 4) swL[4 * q + l] = carried ? static_cast<double>(ci[l]) : 0.0;
    float* hi = q ? hi1 : hi0;
    hi[0] = carried ? ci[8 + l] : 0.0f;
    hi[1] = carried ? ci[8 + 64 + l] : 0.0f;
  }
  wave_lds_fence();
  const int nmax = max(nsub0, nsub1) - 1;
#pragma unroll 1
  for (int it = 0; it < ws::SPB * nmax; ++it) {
    const int sub = ws::SPB > 1 ? it >> 1 : it, q = ws::SPB > 1 ? it & 1 : 0;
    const int nsq = q ? nsub1 : nsub0;
    if (sub >= nsq - 1) continue;
    const int f = b + ws::NBK * q;
    const FuRange g = seg(f);
    double sw[4];
    float hist[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) sw[k] = sg::uni(swL[4 * q + k]);
    hist[0] = q ? hi1[0] : hi0[0];
    hist[1] = q ? hi1[1] : hi0[1];
    ws::wait_ge(&Sync[f][0], sub + 1, a.err);
    const float* PhA = Ring[f][(2 * sub) % 3];
    const float* PhB = Ring[f][(2 * sub + 1) % 3];
    if (ORION_WS_ABL & 1) {
      if (l == 0) ws::lds_st(&Sync[f][1], sub + 1);
    } else {
      ws::job(a, Bc, g, sub, false, PhA, PhB, P, l, sw, hist, &Sync[f][1]);
    }
    if (sub == nsq - 2) {  // the stream's last sub-range is its own wave's: park the state
      float* park = Ring[f][(2 * sub + 4) % 3];
      park[l] = hist[0];
      park[64 + l] = hist[1];
      if (l < 4) reinterpret_cast<double*>(park + 128)[l] = sw[l & 3];
      wave_lds_fence();
      if (l == 0) ws::lds_st(&Sync[f][2], 1);
    } else {
      if (l < 4) swL[4 * q + l] = sw[l & 3];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        hi0[k] = q ? hi0[k] : hist[k];
        hi1[k] = q ? hist[k] : hi1[k];
      }
      wave_lds_fence();
    }
  }
}
}  // namespace

namespace {

constexpr int kFrontR = 2;

// Wave ranges for the wave-independent front: as many resident waves as LDS and
// registers allow, rounded down to a multiple of 4 per CU (one per SIMD each, so
// no SIMD carries more waves than another), one round; each wave owns N tiles =
// N*TW - 1 phi outputs.
struct Front2Plan {
  int grid, wpc;
  long long L;
};
template <int R>
Front2Plan front2_plan(long long n_dec, int nch, int ncu) {
  using G = Fw<R>;
  int per_cu = std::min<int>((160 * 1024) / static_cast<int>(G::LDS_F2 * sizeof(f2)), R <= 2 ? 12 : 8);
  if (const char* e = std::getenv("ORION_WBFM_WPCU")) per_cu = std::atoi(e);  // experiments
  per_cu = std::max(4, per_cu & ~3);
  const long long slots = static_cast<long long>(per_cu) * ncu;
  const long long tiles = static_cast<long long>(nch) * ((n_dec + G::TW) / G::TW);
  long long N = std::max<long long>(1, (tiles + slots - 1) / slots);
  if (const char* e = std::getenv("ORION_WBFM_TILES")) N = std::max(1, std::atoi(e));  // experiments
  Front2Plan p;
  p.L = N * G::TW - 1;
  p.wpc = static_cast<int>((n_dec + p.L - 1) / p.L);
  p.grid = p.wpc * nch;
  return p;
}

template <int R>
void launch_front2(bool a16, long long n_dec, int nch, int ncu, const WbfmArgs& a,
                   const WbfmFrontConst& f, hipStream_t s) {
  const Front2Plan fp = front2_plan<R>(n_dec, nch, ncu);
  if (a.n < 2LL * Fw<R>::NEW) {  // small input: per-lane clamped loads
    if (a16) k_wbfm_front2<R, true, 0, true><<<fp.grid, 64, 0, s>>>(a, f, fp.L, fp.wpc);
    else k_wbfm_front2<R, false, 0, true><<<fp.grid, 64, 0, s>>>(a, f, fp.L, fp.wpc);
  } else {
    if (a16) k_wbfm_front2<R, true, 0><<<fp.grid, 64, 0, s>>>(a, f, fp.L, fp.wpc);
    else k_wbfm_front2<R, false, 0><<<fp.grid, 64, 0, s>>>(a, f, fp.L, fp.wpc);
  }
}

}  // namespace

long long wbfm_fused_slots(long long n_dec, int nch) {
  return static_cast<long long>(nch) * ((n_dec + kFuL - 1) / kFuL) + 1;
}

long long wbfm_seg_slots(long long n_dec, int nch) {
  return static_cast<long long>(nch) * ((n_dec + kSgL - 1) / kSgL) + 1;
}

// One round: as many segments as resident waves (per channel: the channel's share,
// at least one sub-range per segment), each a whole number of sub-ranges.
void launch_wbfm_seg(const WbfmArgs& a, const WbfmFrontConst& f, const WbfmFusedConst& b, int nch,
                     int max_segments, int variant, hipStream_t s) {
  static_assert(sg::L == kSgL && sg2::L == kSgL, "sub-range geometry");
  if (a.n_dec <= 0 || nch <= 0) return;
  static int caps[4] = {0, 0, 0, 0};
  int& cap = caps[variant];
  if (cap == 0) {
    int per_cu = 0, dev = 0, ncu = 0;
    if (variant == 2) ORION_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_wbfm_seg3<true, false>, 64, 0));
    else if (variant == 3) ORION_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_wbfm_seg4<true, false, kSeg4X>, 64, 0));
    else ORION_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_wbfm_seg2<true, false>, 64, 0));
    ORION_HIP(hipGetDevice(&dev));
    ORION_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    cap = std::max(1, per_cu) * std::max(1, ncu);
  }
  const long long capx = max_segments > 0 ? max_segments : cap;
  const long long nsub_ch = (a.n_dec + kSgL - 1) / kSgL;
  // at most the resident capacity (k_wbfm_seg2's end waits on a later segment)
  long long spc = std::max<long long>(1, std::min<long long>(capx / nch, nsub_ch));
  const long long S = (nsub_ch + spc - 1) / spc * kSgL;
  spc = (a.n_dec + S - 1) / S;
  const long long grid = spc * nch;
  if (grid > (1LL << 31) - 1 || S > (1LL << 30)) throw HipError("WBFM segment geometry out of range");
  const bool a16 = (reinterpret_cast<uintptr_t>(a.x) % 16 == 0) && (a.x_stride % 2 == 0);
  const bool clamp = a.n < 2LL * Fw<2>::NEW;
  const int gi = static_cast<int>(grid), sp = static_cast<int>(spc), Si = static_cast<int>(S);
#define ORION_SEG(K)                                                   \
  if (clamp) {                                                         \
    if (a16) K<true, true><<<gi, 64, 0, s>>>(a, f, b, sp, Si);         \
    else K<false, true><<<gi, 64, 0, s>>>(a, f, b, sp, Si);            \
  } else {                                                             \
    if (a16) K<true, false><<<gi, 64, 0, s>>>(a, f, b, sp, Si);        \
    else K<false, false><<<gi, 64, 0, s>>>(a, f, b, sp, Si);           \
  }
  static const int seg4x_env = [] {  // timing experiments: the seg4 variant bits (kSeg4XAlt)
    const char* e = std::getenv("ORION_SEG4_X");
    return e ? std::atoi(e) : -1;
  }();
  const char* ex = std::getenv("ORION_SEG4_X_LIVE");  // in-process A/B (tools/ab_paths.py)
  const int seg4x = ex ? std::atoi(ex) : seg4x_env;
#define ORION_SEG4(XV)                                                         \
  if (clamp) {                                                                 \
    if (a16) k_wbfm_seg4<true, true, XV><<<gi, 64, 0, s>>>(a, f, b, sp, Si);   \
    else k_wbfm_seg4<false, true, XV><<<gi, 64, 0, s>>>(a, f, b, sp, Si);      \
  } else {                                                                     \
    if (a16) k_wbfm_seg4<true, false, XV><<<gi, 64, 0, s>>>(a, f, b, sp, Si);  \
    else k_wbfm_seg4<false, false, XV><<<gi, 64, 0, s>>>(a, f, b, sp, Si);     \
  }
  if (variant == 3 && kSeg4XAlt != kSeg4X && seg4x == kSeg4XAlt) { ORION_SEG4(kSeg4XAlt) } else
  if (variant == 3) { ORION_SEG4(kSeg4X) } else if (variant == 2) { ORION_SEG(k_wbfm_seg3) } else if (variant == 1) { ORION_SEG(k_wbfm_seg2) } else { ORION_SEG(k_wbfm_seg) }
#undef ORION_SEG
#undef ORION_SEG4
  ORION_LAUNCH_CHECK();
}

// k_wbfm_ws: one workgroup of 8 streaming + 4 back waves per CU, one round; the
// segments as in launch_wbfm_seg with 8 per workgroup.
void launch_wbfm_ws(const WbfmArgs& a, const WbfmFrontConst& f, const WbfmFusedConst& b, int nch,
                    int max_segments, hipStream_t s) {
  if (a.n_dec <= 0 || nch <= 0) return;
  constexpr int kThreads = ws::kThreads;
  static int cap = 0;
  if (cap == 0) {
    int per_cu = 0, dev = 0, ncu = 0;
    ORION_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_wbfm_ws<true, false>, kThreads, 0));
    ORION_HIP(hipGetDevice(&dev));
    ORION_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    cap = std::max(1, per_cu) * std::max(1, ncu) * ws::NFR;
  }
  const long long capx = max_segments > 0 ? std::min<long long>(max_segments, cap) : cap;
  const long long nsub_ch = (a.n_dec + kSgL - 1) / kSgL;
  long long spc = std::max<long long>(1, std::min<long long>(capx / nch, nsub_ch));
  const long long S = (nsub_ch + spc - 1) / spc * kSgL;
  spc = (a.n_dec + S - 1) / S;
  const long long nseg = spc * nch;
  // every segment's workgroup is resident at once (a back wave waits on its successor)
  if (nseg > cap) throw HipError("WBFM: more segments than resident waves (too many channels)");
  if (S > (1LL << 30)) throw HipError("WBFM segment geometry out of range");
  const int grid = static_cast<int>((nseg + ws::NFR - 1) / ws::NFR);
  const bool a16 = (reinterpret_cast<uintptr_t>(a.x) % 16 == 0) && (a.x_stride % 2 == 0);
  const bool clamp = a.n < 2LL * Fw<2>::NEW;
  const int sp = static_cast<int>(spc), Si = static_cast<int>(S), ns = static_cast<int>(nseg);
  if (clamp) {
    if (a16) k_wbfm_ws<true, true><<<grid, kThreads, 0, s>>>(a, f, b, sp, Si, ns);
    else k_wbfm_ws<false, true><<<grid, kThreads, 0, s>>>(a, f, b, sp, Si, ns);
  } else {
    if (a16) k_wbfm_ws<true, false><<<grid, kThreads, 0, s>>>(a, f, b, sp, Si, ns);
    else k_wbfm_ws<false, false><<<grid, kThreads, 0, s>>>(a, f, b, sp, Si, ns);
  }
  ORION_LAUNCH_CHECK();
}

void launch_wbfm_fused(const WbfmArgs& a, const WbfmFrontConst& f, const WbfmFusedConst& b, int nch,
                       hipStream_t s) {
  if (a.n_dec <= 0 || nch <= 0) return;
  const bool a16 = (reinterpret_cast<uintptr_t>(a.x) % 16 == 0) && (a.x_stride % 2 == 0);
  const int wpc = static_cast<int>((a.n_dec + kFuL - 1) / kFuL);
  const int grid = wpc * nch;
  static const int kernel = [] {  // 1: one wave per range, 3: persistent (experiments)
    const char* e = std::getenv("ORION_WBFM_KERNEL");
    return e ? std::atoi(e) : 1;
  }();
  int g1 = grid;
  // experiments only: dynamic LDS padding per wave (caps the waves per CU)
  static const int dyn = [] {
    const char* e = std::getenv("ORION_WBFM_DYNLDS");
    return e ? std::atoi(e) : 0;
  }();
  if (kernel == 3) {  // persistent single-role: at most the resident capacity
    static int cap = 0;
    if (cap == 0) {
      int per_cu = 0, dev = 0, ncu = 0;
      ORION_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_wbfm_fused<kFuN, true, false, true>, 64, dyn));
      ORION_HIP(hipGetDevice(&dev));
      ORION_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
      cap = std::max(1, per_cu) * std::max(1, ncu);
    }
    g1 = std::min(grid, cap);
  }
  const bool clamp = a.n < 2LL * Fw<2>::NEW;
  const bool pers = g1 < grid;
#define ORION_FU(A, C, P) k_wbfm_fused<kFuN, A, C, P><<<g1, 64, dyn, s>>>(a, f, b, wpc, grid)
  if (pers) {
    if (clamp) { if (a16) ORION_FU(true, true, true); else ORION_FU(false, true, true); }
    else { if (a16) ORION_FU(true, false, true); else ORION_FU(false, false, true); }
  } else {
    if (clamp) { if (a16) ORION_FU(true, true, false); else ORION_FU(false, true, false); }
    else { if (a16) ORION_FU(true, false, false); else ORION_FU(false, false, false); }
  }
#undef ORION_FU
  ORION_LAUNCH_CHECK();
}

int device_cus() {
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) ncu = p.multiProcessorCount;
  }
  return ncu;
}

void launch_wbfm(const WbfmArgs& a, const WbfmFrontConst& f, const WbfmBackConst& b, int nch,
                 hipStream_t s) {
  if (a.n_dec <= 0 || nch <= 0) return;
  static const int ncu = device_cus();
  const bool a16 = (reinterpret_cast<uintptr_t>(a.x) % 16 == 0) && (a.x_stride % 2 == 0);
  const dim3 gb(div_up(a.n_dec, kBackA), nch);
  launch_front2<kFrontR>(a16, a.n_dec, nch, ncu, a, f, s);
  k_wbfm_back<0><<<gb, NT, 0, s>>>(a, b);
  ORION_LAUNCH_CHECK();
}

}  // namespace orion
