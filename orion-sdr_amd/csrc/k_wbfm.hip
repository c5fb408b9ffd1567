// k_wbfm.hip — fused WBFM demodulation chain for gfx950 (the north-star path).
//
// Reference composition (docs/demodulate.md:128-133, SURVEY §3 stack 2):
//   Rotator(-f_off).rotate_block -> FirDecimator(fs, 8, ...)   (dsp/decim.rs:44-76)
//   -> FmQuadratureDemod (demodulate/fm.rs:45-77) -> FirLowpass (dsp/fir.rs:47-66).
//
// One workgroup (256 threads, 4 waves) owns A consecutive audio outputs and
// streams its input once from HBM in sub-tiles of T = 512 decimated outputs
// (4224 cf32 inputs incl. the 128-sample FIR halo):
//   1. stage: 16-B global loads (prefetched one sub-tile ahead into registers),
//      NCO mix with a per-position phasor table held in registers, scatter into
//      the polyphase LDS image (poly.hpp);
//   2. decim: polyphase FIR at the kept outputs only (2 per lane, packed FMA);
//      the sub-tile's common phasor factor e^{j theta (k0+P_org+1)} is applied
//      to the decimated outputs (linearity: 1 complex mul per 8 inputs);
//   3. discriminator (fm.rs:62-68, atan2_approx op for op) -> LDS;
//   4. LpCascade on wave 0: 8 samples per lane, Kogge-Stone state-carry scan
//      (iir.hpp), re-run with the reference's TDF-II update -> LDS ring;
//   5. audio FIR (2 outputs per lane) -> coalesced stores.
// Across workgroups the IIR state is re-derived by a warm-up of `wpre` outputs
// (pole radius 0.953: transient < 1e-8 relative after 512 samples; the audio
// FIR needs 127 more). The first workgroup of a call starts from the exact state
// carried from the previous call (IIR state, last decimated sample, last 128
// IIR outputs, last 128 raw inputs), so streaming in k calls equals one call.
#include "iir.hpp"
#include "kernels.hpp"
#include "poly.hpp"

namespace orion {
namespace {

constexpr int NT = 256;
constexpr int T = kWbfmT;
constexpr int M = kWbfmM;
constexpr int Q = kWbfmQ;
constexpr int RING = 1024;
using PW = Poly<M, Q, T, NT>;
static_assert(PW::NS == kWbfmNS, "staging size");
constexpr int KP = (PW::NS + 2 * NT - 1) / (2 * NT);  // staged pairs per thread (9)

__device__ __forceinline__ float lp4_step(const BiquadK& bq, float (&s)[4], float x) {
  const float y0 = bq.step(s[0], s[1], x);
  return bq.step(s[2], s[3], y0);
}

template <bool A16>
__global__ __launch_bounds__(NT, 3) void k_wbfm(const WbfmArgs args, const WbfmConst C) {
  __shared__ __attribute__((aligned(16))) f2 U[PW::LDS_F2];
  __shared__ __attribute__((aligned(16))) f2 D[T + 2];
  __shared__ __attribute__((aligned(16))) float ph[T];
  __shared__ __attribute__((aligned(16))) float ring[RING];

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int ch = blockIdx.y;
  const long long n = args.n;
  const long long n_dec = args.n_dec;
  const long long a0 = static_cast<long long>(blockIdx.x) * args.A;
  if (a0 >= n_dec) return;
  const long long a_end = min(a0 + static_cast<long long>(args.A), n_dec);
  long long J0 = a0 - args.wpre;
  const bool first = J0 <= 0;
  if (first) J0 = 0;

  const f2* __restrict__ x = args.x + ch * args.x_stride;
  float* __restrict__ y = args.y + ch * args.y_stride;
  const f2* __restrict__ hist_in = args.hist_in + ch * kWbfmHist;
  const float* __restrict__ carry_in = args.carry_in + ch * kWbfmCarry;
  const uint64_t step = args.step[ch];
  const f2* __restrict__ tab = args.tab + static_cast<long long>(ch) * PW::NS;
  const BiquadK bq{C.b0, C.b1, C.b2, C.a1, C.a2};

  float carry[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  f2 prev = f2{1.0f, 0.0f};
  bool prev_valid = false;
  if (first) {
#pragma unroll
    for (int i = 0; i < 4; ++i) carry[i] = carry_in[i];
    prev = f2{carry_in[4], carry_in[5]};
    prev_valid = true;
    if (t < 128) ring[(t - 128) & (RING - 1)] = carry_in[8 + t];
  }

  f2 pf[KP][2];
  auto prefetch = [&](long long J) {
    const long long porg = static_cast<long long>(M) * (J - Q);
    if (porg >= 0 && porg + PW::NS <= n) {  // interior sub-tile: plain 16-B loads
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        const int p = 2 * t + 2 * NT * k;
        if (p < PW::NS) {
          if constexpr (A16) {
            const f4 v = *reinterpret_cast<const f4*>(x + porg + p);
            pf[k][0] = f2{v.x, v.y};
            pf[k][1] = f2{v.z, v.w};
          } else {
            pf[k][0] = x[porg + p];
            pf[k][1] = x[porg + p + 1];
          }
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        const int p = 2 * t + 2 * NT * k;
        if (p < PW::NS) {
          pf[k][0] = load_hist(x, n, hist_in, kWbfmHist, porg + p);
          pf[k][1] = load_hist(x, n, hist_in, kWbfmHist, porg + p + 1);
        }
      }
    }
  };
  prefetch(J0);

  for (long long J = J0; J < a_end; J += T) {
    // ---- 1. stage (NCO mix, polyphase scatter) ----
    const long long porg = static_cast<long long>(M) * (J - Q);
    const f2 S = phasor_q64(static_cast<uint64_t>(args.k0 + porg + 1), step);
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const int p = 2 * t + 2 * NT * k;
      if (p < PW::NS) {
        // e^{j theta p}, e^{j theta (p+1)}: per-channel table, L2-resident
        const f4 tv = *reinterpret_cast<const f4*>(tab + p);
        U[PW::slot(p)] = cmul_rot(pf[k][0], f2{tv.x, tv.y});
        U[PW::slot(p + 1)] = cmul_rot(pf[k][1], f2{tv.z, tv.w});
      }
    }
    if (J + T < a_end) prefetch(J + T);
    __syncthreads();

    // ---- 2. decimating FIR at the kept outputs ----
    {
      f2 acc[PW::R];
      PW::compute(U, t, [&](int c, int q) { return C.g[c * Q + q]; }, acc);
      const f2 d0 = cmul(acc[0], S);
      const f2 d1 = cmul(acc[1], S);
      D[1 + 2 * t] = d0;
      D[2 + 2 * t] = d1;
      if (t == 0) D[0] = prev_valid ? prev : d0;  // warm-up start: phi = 0
    }
    __syncthreads();

    // ---- 3. FM discriminator (fm.rs:60-68) ----
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int jl = 2 * t + r;
      ph[jl] = fm_disc(D[jl + 1], D[jl], C.k);
    }
    {
      const long long vrem = a_end - J;  // last decimated sample of this sub-tile
      prev = D[vrem < T ? static_cast<int>(vrem) : T];
    }
    prev_valid = true;
    __syncthreads();

    // ---- 4. LpCascade: state-carry scan on wave 0 ----
    if (wave == 0) {
      const long long vrem = a_end - J;
      const int V = vrem < T ? static_cast<int>(vrem) : T;
      float xs[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) xs[i] = ph[8 * lane + i];
      float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (8 * lane + i < V) (void)lp4_step(bq, s, xs[i]);
      if (lane == 0) matvec_acc<4>(C.m8, carry, s);
      wave_scan_inclusive<4>(s, C.pw, lane);
      float e[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float o = __shfl_up(s[i], 1, 64);
        e[i] = lane == 0 ? carry[i] : o;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int jl = 8 * lane + i;
        if (jl < V) ring[(J + jl) & (RING - 1)] = lp4_step(bq, e, xs[i]);
      }
      const int lv = (V - 1) >> 3;
#pragma unroll
      for (int i = 0; i < 4; ++i) carry[i] = __shfl(e[i], lv, 64);
    }
    __syncthreads();

    // ---- 5. audio FIR (fir.rs:57-66, quirk-mapped taps) ----
    {
      const long long jg = J + 2 * t;
      const bool v0 = jg >= a0 && jg < a_end;
      const bool v1 = jg + 1 >= a0 && jg + 1 < a_end;
      if (v0 || v1) {
        float acc0 = 0.0f, acc1 = 0.0f;
        fir2_blocked<128>(
            [&](long long i, float& w0, float& w1) {  // even i: pair never straddles the wrap
              const f2 w = *reinterpret_cast<const f2*>(ring + (i & (RING - 1)));
              w0 = w.x;
              w1 = w.y;
            },
            jg, [&](int k) { return C.a[k]; }, acc0, acc1);
        if (v0) y[jg] = acc0;
        if (v1) y[jg + 1] = acc1;
      }
    }
  }

  // ---- carried state for the next call (workgroup holding the last output) ----
  if (a_end == n_dec) {
    float* __restrict__ carry_out = args.carry_out + ch * kWbfmCarry;
    f2* __restrict__ hist_out = args.hist_out + ch * kWbfmHist;
    if (t == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) carry_out[i] = carry[i];
      carry_out[4] = prev.x;
      carry_out[5] = prev.y;
      carry_out[6] = 0.0f;
      carry_out[7] = 0.0f;
    }
    if (t < 128) {
      carry_out[8 + t] = ring[(n_dec - 128 + t) & (RING - 1)];
      hist_out[t] = load_hist(x, n, hist_in, kWbfmHist, n - 128 + t);
    }
  }
}

}  // namespace

void launch_wbfm(const WbfmArgs& a, const WbfmConst& c, int nch, hipStream_t s) {
  if (a.n_dec <= 0 || nch <= 0) return;
  const dim3 grid(div_up(a.n_dec, a.A), nch);
  const bool a16 = (reinterpret_cast<uintptr_t>(a.x) % 16 == 0) && (a.x_stride % 2 == 0);
  if (a16)
    k_wbfm<true><<<grid, NT, 0, s>>>(a, c);
  else
    k_wbfm<false><<<grid, NT, 0, s>>>(a, c);
  ORION_LAUNCH_CHECK();
}

}  // namespace orion
