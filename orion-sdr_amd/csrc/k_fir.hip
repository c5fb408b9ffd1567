// k_fir.hip — standalone NCO and FIR-family kernels for gfx950.
//   Rotator::rotate_block / mix_usb_block   dsp/rotator.rs:74-94
//   FirDecimator::process                   dsp/decim.rs:44-76 (kept outputs only)
//   FirLowpass::process                     dsp/fir.rs:47-66   (real)
//   FirLowpassIq::process / filter_aligned  dsp/fir.rs:229-297 (complex, real taps)
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "kernels.hpp"
#include "poly.hpp"

namespace orion {
namespace {

constexpr int NT = 256;
constexpr int kMaxGrid = 2048;  // memory-bound: cap and grid-stride (2048 = 8 WG per CU)

// ------------------------------------------------------------------ NCO --
// Output i of a call is oscillator output k = k0 + i (hip_common.hpp OscDev): the
// reference's own phasor from the exact table (tail + unrolled cycle, or the exact
// prefix), or beyond it the model (the closed form when there is no table). MODE:
// kRotate rotate_block (FMA form, rotator.rs:80-83), kUsb mix_usb_block (cf32 -> f32,
// rotator.rs:88-94), kNcoMix mix_with_nco (non-FMA product, nco.rs:63-66), kNcoGen
// the phasors themselves (nco.rs:42-58 next_cs, no input).
enum : int { kRotate = 0, kUsb = 1, kNcoMix = 2, kNcoGen = 3 };
constexpr int kRotMinW = 6;          // waves per SIMD k_rotator is compiled for (8: <= 64 VGPRs, 6 B of spills)
constexpr int kFir4TilesPerCu = 4;   // k_fir_iq8 with 4 outputs per lane below this many 2048-output tiles per CU
constexpr int kRotHp = 2;            // pairs per thread whose loads a full tile issues together
template <bool A16, int MODE>
__global__ __launch_bounds__(NT, kRotMinW) void k_rotator(const f2* __restrict__ x, void* __restrict__ yv, long long n,
                                                uint64_t k0, const OscDev o) {
  constexpr int PER = kRotTile / (2 * NT);  // pairs per thread per tile (8)
  constexpr int HP = kRotHp;
  const int t = threadIdx.x;
  // output pair P, P + 1 (only P when P + 1 == n) from inputs v0, v1 and phasors p0, p1
  auto emit = [&](long long P, bool full, f2 v0, f2 v1, f2 p0, f2 p1) {
    if constexpr (MODE == kUsb) {
      float* y = static_cast<float*>(yv);
      if (A16 && full) {
        *reinterpret_cast<float2*>(y + P) = float2{__builtin_fmaf(v0.x, p0.x, v0.y * p0.y),
                                                   __builtin_fmaf(v1.x, p1.x, v1.y * p1.y)};
      } else {
        y[P] = __builtin_fmaf(v0.x, p0.x, v0.y * p0.y);
        if (full) y[P + 1] = __builtin_fmaf(v1.x, p1.x, v1.y * p1.y);
      }
    } else {
      f2* y = static_cast<f2*>(yv);
      f2 o0, o1;
      if constexpr (MODE == kRotate) {
        o0 = cmul_rot(v0, p0);
        o1 = cmul_rot(v1, p1);
      } else if constexpr (MODE == kNcoMix) {  // (x.re c - x.im s, x.re s + x.im c), no FMA
        o0 = f2{v0.x * p0.x - v0.y * p0.y, v0.x * p0.y + v0.y * p0.x};
        o1 = f2{v1.x * p1.x - v1.y * p1.y, v1.x * p1.y + v1.y * p1.x};
      } else {
        o0 = p0;
        o1 = p1;
      }
      if (A16 && full) {
        *reinterpret_cast<f4*>(y + P) = f4{o0.x, o0.y, o1.x, o1.y};
      } else {
        y[P] = o0;
        if (full) y[P + 1] = o1;
      }
    }
  };
  for (long long tile = static_cast<long long>(blockIdx.x) * kRotTile; tile < n;
       tile += static_cast<long long>(gridDim.x) * kRotTile) {
    const OscRun r = osc_run(o, k0 + static_cast<uint64_t>(tile), kRotTile);  // tile-uniform
    // ld2: the raw reads of a pair's phasors (table entries or mtab), fin2: the phasors
    auto body = [&](auto ld2, auto fin2, auto batched) {
      if (decltype(batched)::value && tile + kRotTile <= n) {  // a full tile, in groups of HP pairs: a group's loads issued together
#pragma unroll
        for (int h = 0; h < PER; h += HP) {
        f2 v0[HP], v1[HP], q0[HP], q1[HP];
#pragma unroll
        for (int i = 0; i < HP; ++i) {
          const int off = 2 * t + 2 * NT * (h + i);
          const long long P = tile + off;
          v0[i] = v1[i] = f2{0.0f, 0.0f};
          if constexpr (MODE != kNcoGen) {
            if (A16) {
              const f4 v = *reinterpret_cast<const f4*>(x + P);
              v0[i] = f2{v.x, v.y};
              v1[i] = f2{v.z, v.w};
            } else {
              v0[i] = x[P];
              v1[i] = x[P + 1];
            }
          }
          ld2(off, q0[i], q1[i]);
        }
#pragma unroll
        for (int i = 0; i < HP; ++i) {
          const int off = 2 * t + 2 * NT * (h + i);
          fin2(off, q0[i], q1[i]);
          emit(tile + off, true, v0[i], v1[i], q0[i], q1[i]);
        }
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int off = 2 * t + 2 * NT * i;
        const long long P = tile + off;
        if (P >= n) break;
        f2 v0 = f2{0.0f, 0.0f}, v1 = f2{0.0f, 0.0f};
        const bool full = P + 1 < n;
        if constexpr (MODE != kNcoGen) {
          v0 = x[P];
          if (full) v1 = x[P + 1];
        }
        f2 p0, p1;
        ld2(off, p0, p1);
        fin2(off, p0, p1);
        emit(P, full, v0, v1, p0, p1);
      }
    };
    auto none = [](int, f2&, f2&) {};
    if (r.kind == 0 && (r.j & 1u) == 0) {  // a 16-B load per pair (the table is padded: no wrap)
      body([&](int off, f2& p0, f2& p1) {
        const f4 v = *reinterpret_cast<const f4*>(o.tab + r.j + off);
        p0 = f2{v.x, v.y};
        p1 = f2{v.z, v.w};
      }, none, std::true_type{});
    } else if (r.kind == 0) {
      body([&](int off, f2& p0, f2& p1) {
        p0 = osc_tab(o, r, off);
        p1 = osc_tab(o, r, off + 1);
      }, none, std::true_type{});
    } else if (r.kind == 1) {
      body([&](int off, f2& p0, f2& p1) {
        const f4 m = *reinterpret_cast<const f4*>(o.mtab + off);
        p0 = f2{m.x, m.y};
        p1 = f2{m.z, m.w};
      }, [&](int off, f2& p0, f2& p1) {
        p0 = osc_model(o, r, off, p0);
        p1 = osc_model(o, r, off + 1, p1);
      }, std::true_type{});
    } else {
      body([&](int off, f2& p0, f2& p1) {
        p0 = osc_ld(o, r, off);
        p1 = osc_ld(o, r, off + 1);
      }, [&](int off, f2& p0, f2& p1) {
        p0 = osc_fin(o, r, off, p0);
        p1 = osc_fin(o, r, off + 1, p1);
      }, std::false_type{});  // one tile per call at most
    }
  }
}

// ------------------------------------------- wave-independent decimator ---
// FirDecimator with M = 8 and K <= 8Q taps (C3: 255 taps, Q = 32) in the WBFM
// front's form. One 64-lane wave per contiguous range of decimated outputs of one
// channel (as many waves as are resident, one round), walked in tiles of TW = 128
// outputs / 1024 new inputs. A tile's inputs are prefetched ahead into registers
// (16-B nontemporal loads, dw_load) and scattered into an 8-row polyphase LDS
// image; the image's leading columns are the previous tile's last ones, copied
// inside LDS. No workgroup barriers, so the register prefetch stays in flight.
// Dw<Q>: the tile geometry shared by the decimator kernels below.
template <int Q>
struct Dw {
  static constexpr int TW = 128;         // outputs per tile
  static constexpr int NEW = 8 * TW;     // new inputs per tile
  static constexpr int KL = NEW / 128;   // 2-sample loads per lane per tile
  static constexpr int LR = TW + Q + 2;  // row pitch (2 mod 16)
  static constexpr int LDS_F2 = 8 * LR;
  static constexpr int WIN = (2 + Q) / 2;  // b128 window reads per lane and phase
  static constexpr int HALO = Q + 2;       // columns carried tile to tile
  static_assert(LR % 16 == 2, "row pitch");
};

// New inputs of the tile whose staged sample 0 is x[porg]: x[porg + 8Q + 2l + 128k (+1)].
// CLAMP = false (n >= 2 NEW): the uniform base is clamped into [0, n - NEW];
// boundary tiles are rewritten exactly at staging. CLAMP: per-lane clamp.
template <int Q, bool A16, bool CLAMP>
__device__ __forceinline__ void dw_load(const f2* __restrict__ x, long long n, long long porg, int l,
                                        f2 (&v)[Dw<Q>::KL][2]) {
  const long long B = porg + 8 * Q;
  const f2* __restrict__ xb;
  int lo = 0, hi = 0;
  if constexpr (CLAMP) {
    constexpr long long kSat = 1LL << 30;
    lo = static_cast<int>(max(-B, -kSat));
    hi = static_cast<int>(min(max((n - 2 - B) & ~1LL, -kSat), kSat));
    xb = x + B;
  } else {
    xb = x + min(max(B, 0LL), (n - Dw<Q>::NEW) & ~1LL);
  }
#pragma unroll
  for (int k = 0; k < Dw<Q>::KL; ++k) {
    const int o = CLAMP ? min(max(2 * l + 128 * k, lo), hi) : 2 * l + 128 * k;
    if constexpr (A16) {
      const f4 w = __builtin_nontemporal_load(reinterpret_cast<const f4*>(xb + o));
      v[k][0] = f2{w.x, w.y};
      v[k][1] = f2{w.z, w.w};
    } else {
      v[k][0] = xb[o];
      v[k][1] = xb[o + 1];
    }
  }
}

// The next call's history of channel ch (last hist_len of [hc | xc[0..n)]), written by
// the wave that owns the channel's first output range (one wave, 64 lanes): no separate
// k_hist_update launch. hist_out is the other buffer of the ping-pong pair.
__device__ __forceinline__ void dw_hist_next(const f2* __restrict__ xc, long long n, const f2* __restrict__ hc,
                                             f2* __restrict__ hist_out, int ch, int hist_len, int l) {
  if (hist_out == nullptr) return;
  f2* __restrict__ hn = hist_out + static_cast<long long>(ch) * hist_len;
  for (int i = l; i < hist_len; i += 64) {
    const long long P = n - hist_len + i;
    hn[i] = P >= 0 ? xc[P] : hc[hist_len + P];
  }
}

// ------------------------------------ four-group wave-independent decimator ---
// k_decim_w4<Q>: k_decim_w with the decimator split over the four ds_read_b128
// lane groups of gfx950 (as k_wbfm.hip's fu_tile8): lane group g (A = lanes 0-3,
// 12-15, 20-27; B = 4-11, 16-19, 28-31; C, D = A, B + 32) sums phases 2g and 2g+1
// for EIGHT outputs per lane (8l'..8l'+7, l' = l & 15), Q taps per phase in blocks
// of 16 (12 window + 4 tap ds_read_b128, 128 v_pk_fma_f32 in eight chains per
// block), and two permlane-swap rounds add the four partial sums, leaving each
// lane two outputs (rows 0, 2, 1, 3 own 8l' + {0,1}, {2,3}, {4,5}, {6,7}). Image
// rows carry a 16-B pad after every four 16-B chunks (lane windows 5 chunks
// apart: conflict-free reads), pitch odd (the phase-scattered b64 staging stores
// spread over banks). Per lane and tile (Q = 32): 64 ds_read_b128 against
// k_decim_w's 136. Taps live in LDS (per-lane phases).
// tap blocks unrolled 4 deep in k_decim_w4: their LDS reads overlap the previous block's FMAs
// (1: 0.66 ms on C3, 4: 0.635)
template <int Q>
struct Dw4 {
  static constexpr int TW = 128;
  static constexpr int NEW = 8 * TW;
  static constexpr int KL = NEW / 128;
  static constexpr int HALO = Q + 2;               // entries carried tile to tile
  static constexpr int NCH = (TW + HALO + 1) / 2;  // 16-B chunks of a row in use
  __host__ __device__ static constexpr int pchunk(int c) { return 5 * (c >> 2) + (c & 3); }
  __host__ __device__ static constexpr int slot(int i) { return 2 * pchunk(i >> 1) + (i & 1); }
  static constexpr int PCH = (pchunk(NCH - 1) + 1) | 1;  // row pitch in chunks, odd
  static constexpr int LRS = 2 * PCH;
  static constexpr int LDS_F2 = 8 * LRS;
  static_assert(Q % 16 == 0 && (TW / 2) % 4 == 0, "geometry");
};
__device__ __forceinline__ int dw4_group(int l) {
  const int i = l & 31;
  const bool a = i < 4 || (i >= 12 && i < 16) || (i >= 20 && i < 28);
  return (l >> 5) * 2 + (a ? 0 : 1);
}
__device__ __forceinline__ int dw4_first_out(int l) {
  const int row = l >> 4;
  return 8 * (l & 15) + 2 * (row == 0 ? 0 : row == 2 ? 1 : row == 1 ? 2 : 3);
}

template <int Q, bool A16, bool CLAMP>
__device__ __forceinline__ void dw4_tile(f2* __restrict__ U, const float* __restrict__ Gt, int l, int n,
                                         long long porg, long long J, const f2* __restrict__ xc, long long nx,
                                         const f2* __restrict__ hc, int hist_len, f2 (&v)[Dw4<Q>::KL][2],
                                         long long pforg, int s0, int s1, f2* __restrict__ outc, long long n_out) {
  using D = Dw4<Q>;
  if (n > 0) {  // halo: entries TW .. TW+Q+1 -> 0 .. Q+1 (chunks TW/2 + h -> h)
#pragma unroll
    for (int r2 = 0; r2 < (8 * D::HALO / 2 + 63) / 64; ++r2) {
      const int e = l + 64 * r2;
      if (e < 8 * D::HALO / 2) {
        const int c = e / (D::HALO / 2), h = e - (D::HALO / 2) * c;
        const int dst = c * D::LRS + 2 * D::pchunk(h);
        *reinterpret_cast<f4*>(U + dst) = *reinterpret_cast<const f4*>(U + dst + 2 * D::pchunk(D::TW / 2));
      }
    }
    wave_lds_fence();
  }
#pragma unroll
  for (int k = 0; k < D::KL; ++k) {  // entry i + 16k = slot(i) + 20k
    U[s0 + 20 * k] = v[k][0];
    U[s1 + 20 * k] = v[k][1];
  }
  asm volatile("" ::: "memory");
  dw_load<Q, A16, CLAMP>(xc, nx, pforg, l, v);  // the tile two ahead (unconditional: see fu_tile)
  const bool bnd = porg < 0 || porg + 8LL * (D::TW + Q) > nx;
  if (bnd || n == 0) {
    wave_lds_fence();
#pragma unroll 1
    for (int p = (n == 0 ? 0 : 8 * Q) + l; p < 8 * (D::TW + Q); p += 64) {
      const long long P = porg + p;
      if (p < 8 * Q || !CLAMP || P < 0 || P >= nx) {
        const int c = (-p) & 7;
        U[c * D::LRS + D::slot((p + c) / 8)] = load_hist(xc, nx, hc, hist_len, P);
      }
    }
  }
  wave_lds_fence();
  const int g = dw4_group(l), lp = l & 15;
  f2 d[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) d[r] = f2{0.0f, 0.0f};
#pragma unroll 4
  for (int b = 0; b < 2 * (Q / 16); ++b) {
    const int c = 2 * g + (b & 1), hq = b >> 1;
    // taps 16hq .. 16hq+15 of phase c read window entries from 2 cb, cb = Q/2 - 8 - 8hq chunks
    const int cb = Q / 2 - 8 - 8 * hq;
    const f4* __restrict__ row = reinterpret_cast<const f4*>(U + c * D::LRS) + 5 * lp + 5 * (cb >> 2);
    f4 w[12];
#pragma unroll
    for (int h = 0; h < 12; ++h) w[h] = row[5 * (h >> 2) + (h & 3)];
    const f4* __restrict__ tq = reinterpret_cast<const f4*>(Gt + c * Q + 16 * hq);
    float t[16];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const f4 u = tq[q4];
      t[4 * q4] = u.x;
      t[4 * q4 + 1] = u.y;
      t[4 * q4 + 2] = u.z;
      t[4 * q4 + 3] = u.w;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q)
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int m = r + 16 - q;  // window entry 1 .. 23
        const f4& wc = w[m >> 1];
        d[r] = fma2(splat2(t[q]), (m & 1) ? f2{wc.z, wc.w} : f2{wc.x, wc.y}, d[r]);
      }
  }
  f2 K[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // rows 0<->1, 2<->3: even rows keep outputs 0..3, odd rows 4..7
    const auto sx = __builtin_amdgcn_permlane16_swap(__float_as_uint(d[i].x), __float_as_uint(d[i + 4].x), false, false);
    const auto sy = __builtin_amdgcn_permlane16_swap(__float_as_uint(d[i].y), __float_as_uint(d[i + 4].y), false, false);
    K[i] = f2{__uint_as_float(sx[0]), __uint_as_float(sy[0])} + f2{__uint_as_float(sx[1]), __uint_as_float(sy[1])};
  }
  f2 F[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // halves: rows 0, 1 keep K[0..1], rows 2, 3 K[2..3]
    const auto sx = __builtin_amdgcn_permlane32_swap(__float_as_uint(K[i].x), __float_as_uint(K[i + 2].x), false, false);
    const auto sy = __builtin_amdgcn_permlane32_swap(__float_as_uint(K[i].y), __float_as_uint(K[i + 2].y), false, false);
    F[i] = f2{__uint_as_float(sx[0]), __uint_as_float(sy[0])} + f2{__uint_as_float(sx[1]), __uint_as_float(sy[1])};
  }
  const long long j = J + dw4_first_out(l);
  if (j + 1 < n_out && (reinterpret_cast<uintptr_t>(outc + j) & 15) == 0) {
    __builtin_nontemporal_store(f4{F[0].x, F[0].y, F[1].x, F[1].y}, reinterpret_cast<f4*>(outc + j));
  } else {
    if (j < n_out) outc[j] = F[0];
    if (j + 1 < n_out) outc[j + 1] = F[1];
  }
}

template <int Q, bool A16, bool CLAMP>
__global__ __launch_bounds__(64, 2) void k_decim_w4(const f2* __restrict__ x, long long x_stride, long long n,
                                                   const f2* __restrict__ hist, int hist_len, f2* __restrict__ out,
                                                   long long out_stride, long long n_out, const Taps256 g, int wpc,
                                                   long long L, f2* __restrict__ hist_out = nullptr) {
  using D = Dw4<Q>;
  __shared__ __attribute__((aligned(16))) f2 U[D::LDS_F2];
  __shared__ __attribute__((aligned(16))) float Gt[8 * Q];
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 8 * Q / 64; ++k) Gt[l + 64 * k] = g.g[l + 64 * k];
  const int ch = blockIdx.x / wpc;
  const long long A = static_cast<long long>(blockIdx.x - ch * wpc) * L;
  const long long B = min(A + L, n_out);
  if (A >= B) return;
  const int ntiles = (static_cast<int>((B - A + D::TW - 1) / D::TW) + 1) & ~1;
  const f2* __restrict__ xc = x + ch * x_stride;
  const f2* __restrict__ hc = hist + static_cast<long long>(ch) * hist_len;
  if (A == 0) dw_hist_next(xc, n, hc, hist_out, ch, hist_len, l);
  f2* __restrict__ outc = out + ch * out_stride;
  const int c0 = (-2 * l) & 7, c1 = (-2 * l - 1) & 7;
  const int s0 = c0 * D::LRS + D::slot((8 * Q + 2 * l + c0) / 8);
  const int s1 = c1 * D::LRS + D::slot((8 * Q + 2 * l + 1 + c1) / 8);
  long long porg = 8LL * (A - Q);
  f2 va[D::KL][2], vb[D::KL][2];
  dw_load<Q, A16, CLAMP>(xc, n, porg, l, va);
  dw_load<Q, A16, CLAMP>(xc, n, porg + D::NEW, l, vb);
  const long long dummy = -8LL * Q;
#pragma unroll 1
  for (int t = 0; t < ntiles; t += 2, porg += 2 * D::NEW) {
    const long long J = A + static_cast<long long>(t) * D::TW;
    dw4_tile<Q, A16, CLAMP>(U, Gt, l, t, porg, J, xc, n, hc, hist_len, va,
                            t + 2 < ntiles ? porg + 2 * D::NEW : dummy, s0, s1, outc, B);
    dw4_tile<Q, A16, CLAMP>(U, Gt, l, t + 1, porg + D::NEW, J + D::TW, xc, n, hc, hist_len, vb,
                            t + 3 < ntiles ? porg + 3 * D::NEW : dummy, s0, s1, outc, B);
  }
}

// k_decim_w4 with four waves per workgroup sharing one tap table (LDS per wave 12.9 KB
// + 1 KB of taps per workgroup instead of per wave) and ONE tile of inputs in flight
// per wave (<= 168 VGPRs): three waves per SIMD instead of two. Each wave still walks
// its own range with no barrier after the tap load. 
template <int Q, bool A16, bool CLAMP>
__global__ __launch_bounds__(256, 3) void k_decim_w4q(const f2* __restrict__ x, long long x_stride, long long n,
                                                     const f2* __restrict__ hist, int hist_len, f2* __restrict__ out,
                                                     long long out_stride, long long n_out, const Taps256 g, int wpc,
                                                     long long L, int nranges, f2* __restrict__ hist_out = nullptr) {
  using D = Dw4<Q>;
  __shared__ __attribute__((aligned(16))) f2 U4[4][D::LDS_F2];
  __shared__ __attribute__((aligned(16))) float Gt[8 * Q];
  for (int k = threadIdx.x; k < 8 * Q; k += 256) Gt[k] = g.g[k];
  __syncthreads();
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = static_cast<int>(blockIdx.x) * 4 + w;
  if (r >= nranges) return;
  f2* __restrict__ U = U4[w];
  const int ch = r / wpc;
  const long long A = static_cast<long long>(r - ch * wpc) * L;
  const long long B = min(A + L, n_out);
  if (A >= B) return;
  const int ntiles = static_cast<int>((B - A + D::TW - 1) / D::TW);
  const f2* __restrict__ xc = x + ch * x_stride;
  const f2* __restrict__ hc = hist + static_cast<long long>(ch) * hist_len;
  if (A == 0) dw_hist_next(xc, n, hc, hist_out, ch, hist_len, l);
  f2* __restrict__ outc = out + ch * out_stride;
  const int c0 = (-2 * l) & 7, c1 = (-2 * l - 1) & 7;
  const int s0 = c0 * D::LRS + D::slot((8 * Q + 2 * l + c0) / 8);
  const int s1 = c1 * D::LRS + D::slot((8 * Q + 2 * l + 1 + c1) / 8);
  long long porg = 8LL * (A - Q);
  f2 va[D::KL][2];
  dw_load<Q, A16, CLAMP>(xc, n, porg, l, va);
  const long long dummy = -8LL * Q;
#pragma unroll 1
  for (int t = 0; t < ntiles; ++t, porg += D::NEW) {
    const long long J = A + static_cast<long long>(t) * D::TW;
    dw4_tile<Q, A16, CLAMP>(U, Gt, l, t, porg, J, xc, n, hc, hist_len, va, t + 1 < ntiles ? porg + D::NEW : dummy,
                            s0, s1, outc, B);
  }
}

__global__ __launch_bounds__(NT) void k_decim_generic(const f2* __restrict__ x, long long x_stride,
                                                      long long n, const f2* __restrict__ hist,
                                                      int hist_len, f2* __restrict__ out,
                                                      long long out_stride, long long n_out, int M,
                                                      int K, const float* __restrict__ g) {
  const int ch = blockIdx.y;
  x += ch * x_stride;
  hist += static_cast<long long>(ch) * hist_len;
  out += ch * out_stride;
  for (long long j = static_cast<long long>(blockIdx.x) * NT + threadIdx.x; j < n_out;
       j += static_cast<long long>(gridDim.x) * NT) {
    f2 acc = f2{0.0f, 0.0f};
    for (int k = 0; k < K; ++k)
      acc = fma2(splat2(g[k]), load_hist(x, n, hist, hist_len, M * j - k), acc);
    out[j] = acc;
  }
}

// The next call's history, fused into the first workgroup of a FIR launch (saves the
// separate k_hist_update launch, ~4 us of a 2^20-sample call): the last hist_len
// samples of [old_h | x[0..n)] into new_h (a different buffer: the histories ping-pong).
template <class V>
__device__ __forceinline__ void hist_next(const V* __restrict__ x, long long n, const V* __restrict__ old_h,
                                          V* __restrict__ new_h, int hist_len) {
  if (new_h == nullptr || blockIdx.x != 0) return;
  for (int i = threadIdx.x; i < hist_len; i += blockDim.x) {
    const long long P = n - hist_len + i;
    new_h[i] = P >= 0 ? x[P] : old_h[hist_len + P];
  }
}

// The FIR's 8-outputs-per-lane block loop over a padded LDS image L (pidx: two slots
// per eight) and LDS taps Gt (k_fir_iq8: complex samples; k_fir_real8: two real halves
// packed). Window base: staged p = pb + 2h, pb = 8 t + KP - 16 kb - 16 (a multiple of 8),
// so pidx(pb + 2h) = 10 (pb / 8) + 2h + 2 (h >> 2): one base per lane, minus 20 per block,
// compile-time offsets (ds_read_b128 with immediates). Output 8 t + r, tap 16 kb + kk
// reads staged p = pb + 16 + r - kk. Per block the taps (wave-uniform LDS reads) come
// first, then the window in the order the FMA chains first need it (tap kk = 0 uses
// entries 16..23, kk = 1 entry 15, ...): LDS reads return in order, so the first FMAs
// wait for 8 reads, not for all 16 and a scalar tap load (lgkmcnt(0)). The summation
// order (kk ascending: the reference's) is unchanged.
template <int KP>
__device__ __forceinline__ void fir8_blocks(const f2* __restrict__ L, const float* __restrict__ Gt, int t,
                                            f2 (&acc)[8]) {
  const f2* __restrict__ Lt = L + 10 * t + 10 * (KP - 16) / 8;
#pragma unroll 1
  for (int kb = 0; kb < KP / 16; ++kb) {
    const f2* __restrict__ Lb = Lt - 20 * kb;
    const f4* __restrict__ tq = reinterpret_cast<const f4*>(Gt + 16 * kb);
    float tp[16];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const f4 u = tq[q4];
      tp[4 * q4] = u.x;
      tp[4 * q4 + 1] = u.y;
      tp[4 * q4 + 2] = u.z;
      tp[4 * q4 + 3] = u.w;
    }
    f2 w[24];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const int h = i < 4 ? 8 + i : 11 - i;  // 8, 9, 10, 11, 7, 6, ..., 0
      const f4 v = *reinterpret_cast<const f4*>(Lb + 2 * h + 2 * (h >> 2));
      w[2 * h] = f2{v.x, v.y};
      w[2 * h + 1] = f2{v.z, v.w};
    }
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const f2 tap = splat2(tp[kk]);
#pragma unroll
      for (int r = 0; r < 8; ++r) acc[r] = fma2(tap, w[16 + r - kk], acc[r]);
    }
  }
}

// Four outputs per lane (small calls: twice the waves of fir8_blocks). Image padded 2
// f2 per 4 samples (pidx4), so lane t's window starts 6t f2 in: the 16 lanes of a
// ds_read_b128 group start 12 banks apart, all distinct. Tap order per output as
// fir8_blocks (bit-identical results).
template <int KP>
__device__ __forceinline__ void fir4_blocks(const f2* __restrict__ L, const float* __restrict__ Gt, int t,
                                            f2 (&acc)[4]) {
  const f2* __restrict__ Lt = L + 6 * t + 3 * (KP - 16) / 2;
#pragma unroll 1
  for (int kb = 0; kb < KP / 16; ++kb) {
    const f2* __restrict__ Lb = Lt - 24 * kb;
    const f4* __restrict__ tq = reinterpret_cast<const f4*>(Gt + 16 * kb);
    float tp[16];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const f4 u = tq[q4];
      tp[4 * q4] = u.x;
      tp[4 * q4 + 1] = u.y;
      tp[4 * q4 + 2] = u.z;
      tp[4 * q4 + 3] = u.w;
    }
    f2 w[20];  // samples p0 .. p0 + 19 (group g of 4 at 6 g)
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int h = i < 2 ? 8 + i : 9 - i;  // the last group first (the first FMAs' operands)
      const f4 v = *reinterpret_cast<const f4*>(Lb + 6 * (h >> 1) + 2 * (h & 1));
      w[2 * h] = f2{v.x, v.y};
      w[2 * h + 1] = f2{v.z, v.w};
    }
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const f2 tap = splat2(tp[kk]);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] = fma2(tap, w[16 + r - kk], acc[r]);
    }
  }
}

// --------------------------------------------------------- real FIR -------
// y[i] = sum_{k<KP} g[k] x[i-k], 512 outputs per sub-tile, 2 per lane.
template <int KP>
__global__ __launch_bounds__(NT) void k_fir_real8(const float* __restrict__ x, long long n,
                                                  const float* __restrict__ hist, int hist_len,
                                                  float* __restrict__ y, const Taps256 g,
                                                  float* __restrict__ hist_out = nullptr) {
  hist_next(x, n, hist, hist_out, hist_len);
  constexpr int TH = 8 * NT, TT = 2 * TH;  // 2048 outputs per half, 4096 per tile
  constexpr int W = TH + KP + 2, PER = (W + NT - 1) / NT;
  constexpr int WP = W + 2 * (W / 8) + 2;
  static_assert(KP % 16 == 0, "taps padded to 16");
  __shared__ __attribute__((aligned(16))) f2 L[WP];
  __shared__ __attribute__((aligned(16))) float Gt[KP];  // the taps (read by the first barrier)
  auto pidx = [](int p) { return p + 2 * (p >> 3); };
  for (int k = threadIdx.x; k < KP; k += NT) Gt[k] = g.g[k];
  auto ld = [&](long long P) {
    float v = 0.0f;
    if (P >= 0) v = P < n ? x[P] : 0.0f;
    else if (P >= -hist_len) v = hist[hist_len + P];
    return v;
  };
  const int t = threadIdx.x;
  for (long long J = static_cast<long long>(blockIdx.x) * TT; J < n; J += static_cast<long long>(gridDim.x) * TT) {
    const long long org = J - KP;  // staged p <-> elements org + p (first half), org + TH + p (second)
    if (org >= 0 && org + TH + W <= n) {  // interior: every load issued before any is used
      float v0[PER], v1[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int p = t + k * NT;
        v0[k] = p < W ? x[org + p] : 0.0f;
        v1[k] = p < W ? x[org + TH + p] : 0.0f;
      }
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int p = t + k * NT;
        if (p < W) L[pidx(p)] = f2{v0[k], v1[k]};
      }
    } else {
      for (int p = t; p < W; p += NT) L[pidx(p)] = f2{ld(org + p), ld(org + TH + p)};
    }
    __syncthreads();
    f2 acc[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = f2{0.0f, 0.0f};
    fir8_blocks<KP>(L, Gt, t, acc);  // as k_fir_iq8 (off = 0), both halves packed
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const long long j0 = J + half * TH + 8 * t;
      float o[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) o[r] = half ? acc[r].y : acc[r].x;
      if (j0 + 8 <= n && (reinterpret_cast<uintptr_t>(y + j0) & 15) == 0) {
        f4* yo = reinterpret_cast<f4*>(y + j0);
        yo[0] = f4{o[0], o[1], o[2], o[3]};
        yo[1] = f4{o[4], o[5], o[6], o[7]};
      } else {
#pragma unroll
        for (int r = 0; r < 8; ++r)
          if (j0 + r < n) y[j0 + r] = o[r];
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(NT) void k_fir_real_generic(const float* __restrict__ x, long long n,
                                                         const float* __restrict__ hist,
                                                         int hist_len, float* __restrict__ y,
                                                         int K, const float* __restrict__ g) {
  for (long long i = static_cast<long long>(blockIdx.x) * NT + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * NT) {
    float acc = 0.0f;
    for (int k = 0; k < K; ++k) {
      const long long P = i - k;
      float v = 0.0f;
      if (P >= 0) v = x[P];
      else if (P >= -hist_len) v = hist[hist_len + P];
      acc = __builtin_fmaf(g[k], v, acc);
    }
    y[i] = acc;
  }
}

// ------------------------------------------------------ complex FIR -------
// y[i] = sum_{k<KP} g[k] x[i-k] on I/Q pairs: a tile of 8*NT outputs, 8 consecutive
// per lane; the tile plus its KP-sample halo is staged once in LDS (padded 2 per 8
// against bank conflicts) behind one barrier. INPLACE (y == x): the halo comes from
// boundary copies E taken before the launch, so no tile reads a neighbour's output.
// Channels (batched FirLowpassIq, independent streams): channel blockIdx.y reads
// x + ch x_stride, writes y + ch y_stride, and keeps its own history at ch hist_len.
template <int KP, bool INPLACE = false, int R = 8>
__global__ __launch_bounds__(NT) void k_fir_iq8(const f2* x, long long n,
                                                const f2* __restrict__ hist, int hist_len,
                                                f2* y, long long n_out, long long off,
                                                const Taps256 g, const f2* __restrict__ E = nullptr,
                                                f2* __restrict__ hist_out = nullptr, long long x_stride = 0,
                                                long long y_stride = 0) {
  if constexpr (!INPLACE) {
    const int ch = blockIdx.y;
    x += ch * x_stride;
    y += ch * y_stride;
    hist += static_cast<long long>(ch) * hist_len;
    if (hist_out) hist_out += static_cast<long long>(ch) * hist_len;
    hist_next(x, n, hist, hist_out, hist_len);
  }
  static_assert(R == 8 || R == 4, "outputs per lane");
  constexpr int TT = R * NT;
  constexpr int W = TT + KP + 2, PER = (W + NT - 1) / NT;
  constexpr int WP = R == 8 ? W + 2 * (W / 8) + 2 : W + 2 * (W / 4) + 2;
  static_assert(KP % 16 == 0, "taps padded to 16");
  __shared__ __attribute__((aligned(16))) f2 L[WP];
  __shared__ __attribute__((aligned(16))) float Gt[KP];  // the taps (read by the first barrier)
  auto pidx = [](int p) { return R == 8 ? p + 2 * (p >> 3) : p + 2 * (p >> 2); };
  const int t = threadIdx.x;
  for (int k = t; k < KP; k += NT) Gt[k] = g.g[k];
  for (long long J = static_cast<long long>(blockIdx.x) * TT; J < n_out;
       J += static_cast<long long>(gridDim.x) * TT) {
    const long long org = J + off - KP;  // staged sample p <-> element org + p
    if constexpr (INPLACE) {
      // halo: HL = J - org samples before the tile, HR = W - HL - TT after it;
      // every load issued before any is used, each from x or the boundary copies
      const long long HL = J - org, HR = W - HL - TT;
      const long long T = J / TT;
      const f2* El = E + T * (HL + HR) - (J - HL);              // El[e], e in [J - HL, J)   (T >= 1)
      const f2* Er = E + (T + 1) * (HL + HR) + HL - (J + TT);   // Er[e], e in [J + TT, ...)
      f2 v[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int p = t + k * NT;
        const long long e = org + p;
        const f2* src = e < J ? El : (e >= J + TT ? Er : x);
        v[k] = (p < W && e >= 0 && e < n) ? src[e] : f2{0.0f, 0.0f};
      }
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int p = t + k * NT;
        if (p < W) L[pidx(p)] = v[k];
      }
    } else if (org >= 0 && org + W <= n) {
      f2 v[PER];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int p = t + k * NT;
        v[k] = p < W ? x[org + p] : f2{0.0f, 0.0f};
      }
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int p = t + k * NT;
        if (p < W) L[pidx(p)] = v[k];
      }
    } else {
      for (int p = t; p < W; p += NT) L[pidx(p)] = load_hist(x, n, hist, hist_len, org + p);
    }
    __syncthreads();
    f2 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = f2{0.0f, 0.0f};
    if constexpr (R == 8) fir8_blocks<KP>(L, Gt, t, acc);
    else fir4_blocks<KP>(L, Gt, t, acc);
    const long long j0 = J + R * t;
    if (j0 + R <= n_out && (reinterpret_cast<uintptr_t>(y + j0) & 15) == 0) {
      f4* yo = reinterpret_cast<f4*>(y + j0);
#pragma unroll
      for (int r = 0; r < R; r += 2) yo[r / 2] = f4{acc[r].x, acc[r].y, acc[r + 1].x, acc[r + 1].y};
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (j0 + r < n_out) y[j0 + r] = acc[r];
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(NT) void k_fir_iq_generic(const f2* __restrict__ x, long long n,
                                                       const f2* __restrict__ hist, int hist_len,
                                                       f2* __restrict__ y, long long n_out,
                                                       long long off, int K,
                                                       const float* __restrict__ g) {
  for (long long i = static_cast<long long>(blockIdx.x) * NT + threadIdx.x; i < n_out;
       i += static_cast<long long>(gridDim.x) * NT) {
    f2 acc = f2{0.0f, 0.0f};
    for (int k = 0; k < K; ++k) acc = fma2(splat2(g[k]), load_hist(x, n, hist, hist_len, i + off - k), acc);
    y[i] = acc;
  }
}

// Boundary copies for the in-place k_fir_iq8: E[b] = x[b TT - HL .. b TT + HR)
// (zeros outside [0, n)), b = 1 .. nb - 1.
__global__ __launch_bounds__(NT) void k_fir_edges(const f2* __restrict__ x, long long n, long long TT, int HL,
                                                  int HR, long long nb, f2* __restrict__ E) {
  const int H = HL + HR;
  for (long long i = static_cast<long long>(blockIdx.x) * NT + threadIdx.x; i < nb * H;
       i += static_cast<long long>(gridDim.x) * NT) {
    const long long b = i / H;
    if (b == 0) continue;
    const long long e = b * TT - HL + (i - b * H);
    E[i] = (e >= 0 && e < n) ? x[e] : f2{0.0f, 0.0f};
  }
}

// History after filter_aligned (fir.rs:266-275 pushes x[0 .. n) then d zeros into
// a reset delay line): h[i] = [x | 0^d][n + d - hist_len + i], zeros before x[0].
__global__ __launch_bounds__(NT) void k_hist_aligned(const f2* __restrict__ x, long long n, long long d,
                                                     int hist_len, f2* __restrict__ h) {
  for (int i = threadIdx.x; i < hist_len; i += NT) {
    const long long P = n + d - hist_len + i;
    h[i] = (P >= 0 && P < n) ? x[P] : f2{0.0f, 0.0f};
  }
}

template <class V>
__global__ void k_hist_update(const V* __restrict__ x, long long n, long long x_stride,
                              const V* __restrict__ old_h, V* __restrict__ new_h, int hist_len) {
  // one workgroup per channel (blockIdx.x): the last hist_len samples of the
  // stream that is this call's input appended to the previous history
  const int ch = blockIdx.x;
  x += ch * x_stride;
  old_h += static_cast<long long>(ch) * hist_len;
  new_h += static_cast<long long>(ch) * hist_len;
  for (int i = threadIdx.x; i < hist_len; i += blockDim.x) {
    const long long P = n - hist_len + i;
    new_h[i] = P >= 0 ? x[P] : old_h[hist_len + P];
  }
}

inline int grid_for(long long work, int per_block) {
  long long g = (work + per_block - 1) / per_block;
  if (g > kMaxGrid) g = kMaxGrid;
  return g < 1 ? 1 : static_cast<int>(g);
}

}  // namespace

void launch_osc(int mode, const f2* x, void* y, long long n, uint64_t k0, const OscDev& o, hipStream_t s) {
  if (n <= 0) return;
  if (o.cyc_len != 0 && o.cyc_len < static_cast<uint64_t>(kOscSpan)) throw HipError("osc: cycle shorter than a run");
  const int grid = grid_for(n, kRotTile);
  const bool a16 = (mode == kNcoGen || reinterpret_cast<uintptr_t>(x) % 16 == 0) &&
                   reinterpret_cast<uintptr_t>(y) % (mode == kUsb ? 8 : 16) == 0;
#define ORION_OSC(MD)                                                                          \
  if (a16) k_rotator<true, MD><<<grid, NT, 0, s>>>(x, y, n, k0, o);                          \
  else k_rotator<false, MD><<<grid, NT, 0, s>>>(x, y, n, k0, o);
  switch (mode) {
    case kRotate: ORION_OSC(kRotate) break;
    case kUsb: ORION_OSC(kUsb) break;
    case kNcoMix: ORION_OSC(kNcoMix) break;
    default: ORION_OSC(kNcoGen) break;
  }
#undef ORION_OSC
  ORION_LAUNCH_CHECK();
}

void launch_decim_batch(const f2* x, long long x_stride, long long n, const f2* hist, int hist_len,
                        f2* out, long long out_stride, long long n_out, int nch, int M, int K,
                        const Taps256& g, const float* g_dev, hipStream_t s, f2* hist_out) {
  if (n_out <= 0 || nch <= 0) return;
  const bool a16 = reinterpret_cast<uintptr_t>(x) % 16 == 0 && x_stride % 2 == 0;
  // M = 8 with 129..256 taps (C3): k_decim_w4q, four waves per workgroup sharing one
  // tap table (three waves per SIMD); M = 8 with <= 128 taps: k_decim_w4.
  if (M == 8 && K > 128 && K <= 256 && hist_len >= 8 * 32) {
    const int capq =
        resident_per_cu(reinterpret_cast<const void*>(k_decim_w4q<32, true, false>), 256) * 4 * device_cus();  // waves
    const long long tiles_ch = (n_out + 127) / 128;
    const long long N = (tiles_ch * nch + capq - 1) / capq;  // tiles per wave
    const long long L = N * 128;
    const long long wpc = (n_out + L - 1) / L;
    const long long nr = wpc * nch;
    if (nr > (1LL << 31) - 1) throw HipError("decimator grid too large");
    const bool clamp = n < 2 * 1024;
    const int gi = static_cast<int>((nr + 3) / 4), wi = static_cast<int>(wpc), ni = static_cast<int>(nr);
    if (clamp) {
      if (a16) k_decim_w4q<32, true, true><<<gi, 256, 0, s>>>(x, x_stride, n, hist, hist_len, out, out_stride, n_out, g, wi, L, ni, hist_out);
      else k_decim_w4q<32, false, true><<<gi, 256, 0, s>>>(x, x_stride, n, hist, hist_len, out, out_stride, n_out, g, wi, L, ni, hist_out);
    } else {
      if (a16) k_decim_w4q<32, true, false><<<gi, 256, 0, s>>>(x, x_stride, n, hist, hist_len, out, out_stride, n_out, g, wi, L, ni, hist_out);
      else k_decim_w4q<32, false, false><<<gi, 256, 0, s>>>(x, x_stride, n, hist, hist_len, out, out_stride, n_out, g, wi, L, ni, hist_out);
    }
    ORION_LAUNCH_CHECK();
    return;
  }
  if (M == 8 && K <= 256 && hist_len >= 8 * (K <= 128 ? 16 : 32)) {
    const int cap = std::max(4, resident_per_cu(reinterpret_cast<const void*>(k_decim_w4<32, true, false>), 64) & ~3) *
                    device_cus();  // a multiple of 4 per CU: balanced SIMDs
    const long long tiles_ch = (n_out + 127) / 128;
    long long N = (tiles_ch * nch + cap - 1) / cap;
    N = (N + 1) & ~1LL;  // tiles per wave, even
    const long long L = N * 128;
    const long long wpc = (n_out + L - 1) / L;
    const long long grid = wpc * nch;
    if (grid > (1LL << 31) - 1) throw HipError("decimator grid too large");
    const bool clamp = n < 2 * 1024;
    const int gi = static_cast<int>(grid), wi = static_cast<int>(wpc);
#define ORION_DW(KK, QQ)                                                                                    \
  if (clamp) {                                                                                              \
    if (a16) KK<QQ, true, true><<<gi, 64, 0, s>>>(x, x_stride, n, hist, hist_len, out, out_stride, n_out, g, wi, L, hist_out); \
    else KK<QQ, false, true><<<gi, 64, 0, s>>>(x, x_stride, n, hist, hist_len, out, out_stride, n_out, g, wi, L, hist_out); \
  } else {                                                                                                  \
    if (a16) KK<QQ, true, false><<<gi, 64, 0, s>>>(x, x_stride, n, hist, hist_len, out, out_stride, n_out, g, wi, L, hist_out); \
    else KK<QQ, false, false><<<gi, 64, 0, s>>>(x, x_stride, n, hist, hist_len, out, out_stride, n_out, g, wi, L, hist_out); \
  }
    if (K <= 128) { ORION_DW(k_decim_w4, 16) } else { ORION_DW(k_decim_w4, 32) }
#undef ORION_DW
  } else {
    const dim3 grid(grid_for(n_out, NT), nch);
    k_decim_generic<<<grid, NT, 0, s>>>(x, x_stride, n, hist, hist_len, out, out_stride, n_out, M, K, g_dev);
    if (hist_out) launch_hist_update_c(x, n, hist, hist_out, hist_len, s, nch, x_stride);
  }
  ORION_LAUNCH_CHECK();
}

void launch_decim(const f2* x, long long n, const f2* hist, int hist_len, f2* out, long long n_out,
                  int M, int K, const Taps256& g, const float* g_dev, hipStream_t s) {
  launch_decim_batch(x, n, n, hist, hist_len, out, n_out, n_out, 1, M, K, g, g_dev, s);
}

void launch_fir_real(const float* x, long long n, const float* hist, int hist_len, float* y, int K,
                     const Taps256& g, const float* g_dev, hipStream_t s, float* hist_out) {
  if (n <= 0) return;
  const int g16 = static_cast<int>(std::min<long long>(kMaxGrid, (n + 16 * NT - 1) / (16 * NT)));
  if (K <= 64 && hist_len >= 64) k_fir_real8<64><<<g16, NT, 0, s>>>(x, n, hist, hist_len, y, g, hist_out);
  else if (K <= 128 && hist_len >= 128) k_fir_real8<128><<<g16, NT, 0, s>>>(x, n, hist, hist_len, y, g, hist_out);
  else if (K <= 256 && hist_len >= 256) k_fir_real8<256><<<g16, NT, 0, s>>>(x, n, hist, hist_len, y, g, hist_out);
  else {
    k_fir_real_generic<<<grid_for(n, NT), NT, 0, s>>>(x, n, hist, hist_len, y, K, g_dev);
    if (hist_out) launch_hist_update_r(x, n, hist, hist_out, hist_len, s);
  }
  ORION_LAUNCH_CHECK();
}

void launch_fir_iq(const f2* x, long long n, const f2* hist, int hist_len, f2* y, long long n_out,
                   long long off, int K, const Taps256& g, const float* g_dev, hipStream_t s, f2* hist_out,
                   int nch, long long x_stride, long long y_stride) {
  if (n_out <= 0 || nch <= 0) return;
  if (K <= 256 && hist_len >= (K <= 64 ? 64 : K <= 128 ? 128 : 256)) {
    // calls that fill fewer than kFir4TilesPerCu tiles of 8 outputs per lane per CU
    // take four outputs per lane (twice the waves; the FMA work is the same)
    const bool four = n_out * nch < static_cast<long long>(kFir4TilesPerCu) * device_cus() * 8 * NT;
    if (four) {
      const dim3 g4(grid_for(n_out, 4 * NT), nch);
      if (K <= 64) k_fir_iq8<64, false, 4><<<g4, NT, 0, s>>>(x, n, hist, hist_len, y, n_out, off, g, nullptr, hist_out, x_stride, y_stride);
      else if (K <= 128) k_fir_iq8<128, false, 4><<<g4, NT, 0, s>>>(x, n, hist, hist_len, y, n_out, off, g, nullptr, hist_out, x_stride, y_stride);
      else k_fir_iq8<256, false, 4><<<g4, NT, 0, s>>>(x, n, hist, hist_len, y, n_out, off, g, nullptr, hist_out, x_stride, y_stride);
    } else {
      const dim3 g8(grid_for(n_out, 8 * NT), nch);
      if (K <= 64) k_fir_iq8<64><<<g8, NT, 0, s>>>(x, n, hist, hist_len, y, n_out, off, g, nullptr, hist_out, x_stride, y_stride);
      else if (K <= 128) k_fir_iq8<128><<<g8, NT, 0, s>>>(x, n, hist, hist_len, y, n_out, off, g, nullptr, hist_out, x_stride, y_stride);
      else k_fir_iq8<256><<<g8, NT, 0, s>>>(x, n, hist, hist_len, y, n_out, off, g, nullptr, hist_out, x_stride, y_stride);
    }
  } else {
    for (int ch = 0; ch < nch; ++ch) {
      const f2* xc = x + ch * x_stride;
      const f2* hc = hist + static_cast<long long>(ch) * hist_len;
      k_fir_iq_generic<<<grid_for(n_out, NT), NT, 0, s>>>(xc, n, hc, hist_len, y + ch * y_stride, n_out, off, K, g_dev);
      if (hist_out) launch_hist_update_c(xc, n, hc, hist_out + static_cast<long long>(ch) * hist_len, hist_len, s);
    }
  }
  ORION_LAUNCH_CHECK();
}

bool launch_fir_iq_aligned_inplace(f2* io, long long n, long long d, int K, const Taps256& g, f2* edges,
                                   long long edges_cap, f2* hist_out, int hist_len, hipStream_t s) {
  if (n <= 0) return true;
  if (K > 256) return false;
  const int KP = K <= 64 ? 64 : K <= 128 ? 128 : 256;
  constexpr long long TT = 8 * NT;
  const long long W = TT + KP + 2;
  const int HL = static_cast<int>(KP - d), HR = static_cast<int>(W - (KP - d) - TT);
  const long long nb = (n + TT - 1) / TT;
  if (nb * (HL + HR) > edges_cap) return false;
  // the history (read before the samples are overwritten), then the boundary copies
  k_hist_aligned<<<1, NT, 0, s>>>(io, n, d, hist_len, hist_out);
  if (nb > 1) k_fir_edges<<<grid_for(nb * (HL + HR), NT), NT, 0, s>>>(io, n, TT, HL, HR, nb, edges);
  const int g8 = grid_for(n, 8 * NT);
  if (KP == 64) k_fir_iq8<64, true><<<g8, NT, 0, s>>>(io, n, nullptr, 0, io, n, d, g, edges);
  else if (KP == 128) k_fir_iq8<128, true><<<g8, NT, 0, s>>>(io, n, nullptr, 0, io, n, d, g, edges);
  else k_fir_iq8<256, true><<<g8, NT, 0, s>>>(io, n, nullptr, 0, io, n, d, g, edges);
  ORION_LAUNCH_CHECK();
  return true;
}
long long fir_iq_aligned_edges(long long n, int K) {
  const int KP = K <= 64 ? 64 : K <= 128 ? 128 : 256;
  const long long TT = 8 * NT, W = TT + KP + 2;
  return ((n + TT - 1) / TT) * (W - TT);
}

void launch_hist_update_c(const f2* x, long long n, const f2* old_h, f2* new_h, int hist_len,
                          hipStream_t s, int nch, long long x_stride) {
  if (hist_len <= 0 || nch <= 0) return;
  k_hist_update<f2><<<nch, NT, 0, s>>>(x, n, x_stride, old_h, new_h, hist_len);
  ORION_LAUNCH_CHECK();
}
void launch_hist_update_r(const float* x, long long n, const float* old_h, float* new_h,
                          int hist_len, hipStream_t s) {
  if (hist_len <= 0) return;
  k_hist_update<float><<<1, NT, 0, s>>>(x, n, n, old_h, new_h, hist_len);
  ORION_LAUNCH_CHECK();
}

namespace {
// e^{j 2 pi k step / 2^64}, k < n (the oscillator model's step table, osc.cpp): the angle
// reduced exactly as a Q0.64 turn count, then an f64 sincos; built on the device at a
// (re)tune instead of on the host (~1-4 ms there) and uploaded
__global__ __launch_bounds__(NT) void k_phasor_q64(f2* __restrict__ out, uint64_t step_q64, int n) {
  const int k = static_cast<int>(blockIdx.x) * NT + static_cast<int>(threadIdx.x);
  if (k >= n) return;
  const uint64_t ph = static_cast<uint64_t>(k) * step_q64;
  const double a = static_cast<double>(static_cast<int64_t>(ph)) * (6.283185307179586476925286766559 / 18446744073709551616.0);
  double sn, cs;
  sincos(a, &sn, &cs);
  out[k] = f2{static_cast<float>(cs), static_cast<float>(sn)};
}
}  // namespace

void launch_phasor_table_q64(f2* out, uint64_t step_q64, int n, hipStream_t s) {
  if (n <= 0) return;
  k_phasor_q64<<<(n + NT - 1) / NT, NT, 0, s>>>(out, step_q64, n);
  ORION_LAUNCH_CHECK();
}

}  // namespace orion
