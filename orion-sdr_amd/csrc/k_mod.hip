// k_mod.hip — on-device analog modulators for gfx950.
//   AmDsbMod::process          modulate/am.rs:44-120
//   PmDirectPhaseMod::process  modulate/pm.rs:36-47
//   FmPhaseAccumMod::process   modulate/fm.rs:45-74 (+ mix_with_nco, dsp/nco.rs:62-66)
//   SsbPhasingMod::process     modulate/ssb.rs:43-114 (front and back of the two
//                              LpCascade scans, which run on the k_scan kernels)
// Every oscillator is the reference's own recurrence (hip_common.hpp OscDev, osc.hpp
// RefOsc): sample i of a call uses oscillator output k0 + i (Rotator::next /
// Nco::next_cs advance before returning) — the tabulated reference phasor, or past the
// table the drift model. Streaming, memory-bound kernels: tiles of kModTile samples
// (one oscillator cursor each), grid-stride, at most 8 workgroups per CU.
#include <algorithm>

#include "kernels.hpp"

namespace orion {
namespace {

constexpr int NT = 256;
constexpr int kMaxGrid = 2048;
constexpr int kFmC = 16;             // FM phase scan: samples per thread
constexpr int kFmCH = kFmC * NT;     // samples per workgroup chunk (4096)

constexpr int kModPer = 8;               // samples per thread per tile
constexpr int kModTile = NT * kModPer;   // 2048
static_assert(kModTile <= kOscSpan, "one oscillator cursor per tile");

int grid_for(long long n) {
  return static_cast<int>(std::min<long long>(kMaxGrid, std::max(1LL, (n + kModTile - 1) / kModTile)));
}

// Sample i of a call with its oscillator phasor (output k0 + i): f(i, ld(i), r). A
// full tile issues the loads of kModGrp samples (input and phasor reads) before it
// uses any (a guarded load per sample waits for itself before the next is issued).
constexpr int kModGrp = 4;
template <class L, class F>
__device__ __forceinline__ void mod_tiles(long long n, uint64_t k0, const OscDev& o, L ld, F f) {
  for (long long tile = static_cast<long long>(blockIdx.x) * kModTile; tile < n;
       tile += static_cast<long long>(gridDim.x) * kModTile) {
    const OscRun r = osc_run(o, k0 + static_cast<uint64_t>(tile), kModTile);
    if (tile + kModTile <= n && r.kind != 2) {
#pragma unroll
      for (int g = 0; g < kModPer; g += kModGrp) {
        decltype(ld(0LL)) v[kModGrp];
        f2 p[kModGrp];
#pragma unroll
        for (int m = 0; m < kModGrp; ++m) {
          const int off = static_cast<int>(threadIdx.x) + NT * (g + m);
          v[m] = ld(tile + off);
          p[m] = osc_ld(o, r, off);
        }
#pragma unroll
        for (int m = 0; m < kModGrp; ++m) {
          const int off = static_cast<int>(threadIdx.x) + NT * (g + m);
          f(tile + off, v[m], osc_fin(o, r, off, p[m]));
        }
      }
      continue;
    }
#pragma unroll
    for (int m = 0; m < kModPer; ++m) {
      const int off = static_cast<int>(threadIdx.x) + NT * m;
      const long long i = tile + off;
      if (i < n) f(i, ld(i), osc_get(o, r, off));
    }
  }
}

// am.rs:87-89 (clamp: :56): m = (cl + mi x) [clamped to +-1] * g; out = m * r (Rotator rf).
__global__ __launch_bounds__(NT) void k_am_mod(const float* __restrict__ x, f2* __restrict__ y, long long n,
                                               uint64_t k0, const OscDev o, float cl, float mi, float g, int clamp) {
  mod_tiles(n, k0, o, [&](long long i) { return x[i]; }, [&](long long i, float xi, f2 r) {
    float v = cl + mi * xi;
    if (clamp) v = fminf(fmaxf(v, -1.0f), 1.0f);
    const float m = v * g;
    y[i] = f2{m * r.x, m * r.y};
  });
}

// modulate/pm.rs:36-47 PmDirectPhaseMod: phi = kp x; base = (cos phi, sin phi) * gain
// (num-complex Complex * f32); out = mix_with_nco(base, rf) (the non-FMA product,
// nco.rs:63-66).
__global__ __launch_bounds__(NT) void k_pm_mod(const float* __restrict__ x, f2* __restrict__ y, long long n,
                                               uint64_t k0, const OscDev o, float kp, float g) {
  mod_tiles(n, k0, o, [&](long long i) { return x[i]; }, [&](long long i, float xi, f2 r) {
    const float phi = kp * xi;
    float sn, cs;
    sincos_cr(phi, &sn, &cs);  // pm.rs:44 (phi.cos(), phi.sin())
    const float br = cs * g, bi = sn * g;
    y[i] = f2{br * r.x - bi * r.y, br * r.y + bi * r.x};
  });
}

// ssb.rs:52-54: the two LpCascade inputs x p.re, x p.im (p = audio NCO), planar.
__global__ __launch_bounds__(NT) void k_ssb_mod_front(const float* __restrict__ x, float* __restrict__ u,
                                                      long long n, uint64_t k0, const OscDev o) {
  mod_tiles(n, k0, o, [&](long long i) { return x[i]; }, [&](long long i, float xi, f2 p) {
    u[i] = xi * p.x;
    u[n + i] = xi * p.y;
  });
}

// ssb.rs:55-60: z = (I, side Q); out = z * r (rf NCO), FMA form of rotate_block.
__global__ __launch_bounds__(NT) void k_ssb_mod_back(const float* __restrict__ v, f2* __restrict__ y, long long n,
                                                     uint64_t k0, const OscDev o, float side) {
  mod_tiles(n, k0, o, [&](long long i) { return f2{v[i], v[n + i]}; }, [&](long long i, f2 vi, f2 r) {
    const f2 z = f2{vi.x, side * vi.y};
    y[i] = cmul_rot(z, r);
  });
}

// ---- FmPhaseAccumMod (fm.rs:45-74) ----------------------------------------------------
// The reference multiplies a running phasor z by the f32 pair (dc, ds) = sin_cos(kf x)
// per sample (renormalising |z| every 1024 samples). The angle of that f32 pair, not
// kf x itself, is what it adds, and the difference is systematic (1.2e-2 rad over 2^20
// samples of the C2 input), so the phase must sum the pairs' own angles. Here:
//   * thread t owns 16 consecutive samples; it forms their pairs, their product in f64
//     and one f64 atan2 of that product: the sum of the 16 angles mod 2 pi, exact to
//     ~1e-16 rad, as a Q0.64 turn count (wrapping uint64);
//   * phases are sums of those counts — exact integer arithmetic, associative, so the
//     prefix over threads, waves and chunks (decoupled look-back) is bit-reproducible
//     in any order and never drifts, and the carried phase is exact mod 2 pi;
//   * the thread's outputs: the phasor of its entering phase (phasor_at), then the
//     reference's own recurrence z = z (dc, ds) (fm.rs:53-54, its op order) over its
//     16 pairs; base = z gain (fm.rs:66); mix_with_nco's non-FMA product with the
//     RF Nco's phasor (nco.rs:62-66; the oscillator cursor of the chunk).
// Against an f64 phase and a per-sample sincosf of it this is ~3x less VALU per sample.
constexpr int kFmLb = 1;    // look-back records per lane and step (64 kFmLb chunks per step)
constexpr int kFmG = 8;     // RF phasor reads per thread issued together
constexpr int kFmMinW = 1;  // waves per SIMD k_fm_mod_sp is compiled for (A/B: 5 = 96 VGPRs was slower)
constexpr double kTurnsPerRad = 2.9358905032820014e18;  // 2^64 / (2 pi)

struct FmPairs {
  float c[kFmC], s[kFmC];
};
// The thread's pairs (fm.rs:50-51) and the Q0.64 sum of their angles; samples past n
// (valid < kFmC) are pairs (1, 0).
// FULL: every thread's kFmC samples are valid (no per-sample test).
template <bool FULL = false>
__device__ __forceinline__ uint64_t fm_pairs(float kf, const float* __restrict__ xs, int valid, FmPairs& p) {
  double pr = 1.0, pi = 0.0;
#pragma unroll
  for (int k = 0; k < kFmC; ++k) {
    float sn = 0.0f, cs = 1.0f;
    if (FULL || k < valid) sincos_cr(kf * xs[k], &sn, &cs);  // fm.rs:50-51
    p.c[k] = cs;
    p.s[k] = sn;
    const double c = cs, s = sn;
    const double nr = __builtin_fma(pr, c, -pi * s);
    pi = __builtin_fma(pr, s, pi * c);
    pr = nr;
  }
  const double th = atan2(pi, pr);  // in [-pi, pi]: the 16 angles' sum mod 2 pi
  // (half turns' count doubled: th = +-pi would overflow an int64 of 2^-64 turns)
  return static_cast<uint64_t>(static_cast<long long>(rint(th * kTurnsPerRad * 0.5))) * 2u;
}

// Outputs of the chunk: thread t's samples i0 .. i0 + 15 (i0 = base + 16 t) from its
// entering phase ph. Each thread writes its 16 base values z gain to LDS (ys, one pad
// slot per 16), then the chunk is mixed with the RF phasors and stored in sample order
// (e = t + 256 m): the stores and the RF table reads are coalesced (a thread's own 16
// consecutive samples would touch 64 cache lines per wave instruction). ys aliases
// the input staging: every thread is past its reads of it (the caller's barrier).
constexpr int kFmYs = kFmCH + kFmCH / 16;  // f2 slots
template <bool FULL = false>
__device__ __forceinline__ void fm_out(const FmPairs& p, uint64_t ph, float gain, const OscDev& o, uint64_t k0,
                                       f2* ys, f2* __restrict__ y, long long base, long long n) {
  const OscRun R = osc_run(o, k0 + static_cast<uint64_t>(base), kFmCH);  // RF Nco outputs of the chunk
  const int t = threadIdx.x;
  f2 z = phasor_at(ph);
#pragma unroll
  for (int k = 0; k < kFmC; ++k) {
    // fm.rs:53-54: zr = z.re.mul_add(dc, -z.im*ds); zi = z.im.mul_add(dc, z.re*ds)
    z = f2{__builtin_fmaf(z.x, p.c[k], -(z.y * p.s[k])), __builtin_fmaf(z.y, p.c[k], z.x * p.s[k])};
    const int e = kFmC * t + k;
    ys[e + (e >> 4)] = f2{z.x * gain, z.y * gain};  // fm.rs:66 base = z * gain
  }
  // the RF phasor reads in groups of G (the first group in flight across the barrier)
  constexpr int G = kFmG;
  const bool full = base + kFmCH <= n;
  f2 rp[G];
  auto rd = [&](int g) {
#pragma unroll
    for (int m = 0; m < G; ++m) rp[m] = osc_ld(o, R, t + NT * (g + m));
  };
  rd(0);
  __syncthreads();
#pragma unroll
  for (int g = 0; g < kFmC; g += G) {
    if (g) rd(g);
#pragma unroll
    for (int m = 0; m < G; ++m) {
      const int e = t + NT * (g + m);
      const f2 bz = ys[e + (e >> 4)];
      const f2 r = osc_fin(o, R, e, rp[m]);
      if (FULL || full || base + e < n) y[base + e] = f2{bz.x * r.x - bz.y * r.y, bz.x * r.y + bz.y * r.x};  // nco.rs:65
    }
  }
}

// Exclusive / inclusive prefix of a uint64 over the workgroup (4 waves); tot: 4 slots.
__device__ __forceinline__ uint64_t u64_up(uint64_t v, int d) {
  const uint32_t lo = __shfl_up(static_cast<uint32_t>(v), d, 64), hi = __shfl_up(static_cast<uint32_t>(v >> 32), d, 64);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}
__device__ __forceinline__ uint64_t wg_scan_u64(uint64_t v, uint64_t* tot, uint64_t& total) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint64_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t o = u64_up(inc, d);
    if (lane >= d) inc += o;
  }
  if (lane == 63) tot[w] = inc;
  __syncthreads();
  uint64_t before = inc - v;
  total = 0;
#pragma unroll
  for (int k = 0; k < NT / 64; ++k) {
    if (k < w) before += tot[k];
    total += tot[k];
  }
  return before;
}

// Coalesced load of the chunk into LDS; thread t then reads its 16 consecutive samples.
// The loads are unconditional (index clamped to n - 1, n >= 1): all 16 in flight at
// once. A guarded load per sample compiles to a branch around each, and each then
// waits for its own load before the LDS store (16 serial memory latencies per chunk).
template <bool FULL = false>
__device__ __forceinline__ int fm_stage(const float* __restrict__ x, long long n, long long base, float* xs) {
  float v[kFmC];
#pragma unroll
  for (int k = 0; k < kFmC; ++k) v[k] = x[FULL ? base + threadIdx.x + k * NT : min(base + threadIdx.x + k * NT, n - 1)];
#pragma unroll
  for (int k = 0; k < kFmC; ++k) {
    const int e = threadIdx.x + k * NT;
    xs[e + (e >> 4)] = FULL || base + e < n ? v[k] : 0.0f;
  }
  __syncthreads();
  const long long i0 = base + static_cast<long long>(threadIdx.x) * kFmC;
  return static_cast<int>(max(0LL, min(static_cast<long long>(kFmC), n - i0)));
}

// Three-pass form (orion_block_configure MOD_PASSES 3). Pass 1: each chunk's Q0.64 sum.
__global__ __launch_bounds__(NT) void k_fm_mod_sum(const float* __restrict__ x, long long n, float kf,
                                                   uint64_t* __restrict__ sums) {
  __shared__ uint64_t tot[NT / 64];
  __shared__ float xs[kFmCH + kFmCH / 16];
  const long long base = static_cast<long long>(blockIdx.x) * kFmCH;
  const int valid = fm_stage(x, n, base, xs);
  FmPairs p;
  const int e = threadIdx.x * kFmC;
  const uint64_t q = fm_pairs(kf, xs + e + (e >> 4), valid, p);
  uint64_t total;
  (void)wg_scan_u64(q, tot, total);
  if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// Pass 2 (one workgroup): exclusive prefix of the chunk sums from the carried phase;
// the carried phase of the next call.
__global__ __launch_bounds__(NT) void k_fm_mod_carry(uint64_t* __restrict__ sums, int nchunk,
                                                     const uint64_t* __restrict__ carry_in,
                                                     uint64_t* __restrict__ carry_out) {
  __shared__ uint64_t tot[NT / 64];
  const int t = threadIdx.x;
  const int per = (nchunk + NT - 1) / NT;
  const int c0 = min(nchunk, t * per), c1 = min(nchunk, c0 + per);
  uint64_t run = 0;
  for (int c = c0; c < c1; ++c) run += sums[c];
  uint64_t total;
  uint64_t before = carry_in[0] + wg_scan_u64(run, tot, total);
  for (int c = c0; c < c1; ++c) {
    const uint64_t v = sums[c];
    sums[c] = before;
    before += v;
  }
  if (t == 0) carry_out[0] = carry_in[0] + total;
}

// Pass 3: the block scan of the thread sums from the chunk's entering phase, outputs.
__global__ __launch_bounds__(NT) void k_fm_mod_apply(const float* __restrict__ x, f2* __restrict__ y, long long n,
                                                     float kf, float gain, const uint64_t* __restrict__ offs,
                                                     uint64_t k0, const OscDev o) {
  __shared__ uint64_t tot[NT / 64];
  __shared__ __attribute__((aligned(16))) f2 ys[kFmYs];  // the input staging, then the outputs
  float* xs = reinterpret_cast<float*>(ys);
  static_assert(2 * kFmYs >= kFmCH + kFmCH / 16, "staging fits");
  const long long base = static_cast<long long>(blockIdx.x) * kFmCH;
  const int valid = fm_stage(x, n, base, xs);
  FmPairs p;
  const int e = threadIdx.x * kFmC;
  const uint64_t q = fm_pairs(kf, xs + e + (e >> 4), valid, p);
  uint64_t total;
  const uint64_t ph = offs[blockIdx.x] + wg_scan_u64(q, tot, total);  // (its barrier: xs is dead)
  fm_out(p, ph, gain, o, k0, ys, y, base, n);
}

// Single pass (default): each chunk publishes its Q0.64 sum, takes the phase entering
// it by decoupled look-back over its predecessors (wave 0: lane i looks at chunk
// c-1-i; the nearest chunk with a published inclusive prefix, or the carried phase
// before chunk 0, closes the sum), then publishes its inclusive prefix. Integer sums:
// the result does not depend on which records the walk found. Chunk-major grid: every
// predecessor was dispatched earlier and publishes its sum before it waits, so the
// walk always ends. Records: 8 u32 per chunk, [0, 2) sum, [2, 4) inclusive prefix,
// 6 / 7 their flags (launch epoch).
__device__ __forceinline__ void fm_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t fm_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void fm_st64(uint32_t* p, uint64_t v) {
  fm_st(p, static_cast<uint32_t>(v));
  fm_st(p + 1, static_cast<uint32_t>(v >> 32));
}
__device__ __forceinline__ uint64_t fm_ld64(const uint32_t* p) {
  return (static_cast<uint64_t>(fm_ld(p + 1)) << 32) | fm_ld(p);
}

__global__ __launch_bounds__(NT, kFmMinW) void k_fm_mod_sp(const float* __restrict__ x, f2* __restrict__ y, long long n,
                                                  float kf, float gain, uint32_t* __restrict__ rec, uint32_t epoch,
                                                  const uint64_t* __restrict__ carry_in, uint64_t* __restrict__ carry_out,
                                                  uint64_t k0, const OscDev o, int* __restrict__ err, uint32_t spin) {
  __shared__ uint64_t tot[NT / 64];
  __shared__ uint64_t excl_sh;
  __shared__ __attribute__((aligned(16))) f2 ys[kFmYs];  // the input staging, then the outputs
  float* xs = reinterpret_cast<float*>(ys);
  static_assert(2 * kFmYs >= kFmCH + kFmCH / 16, "staging fits");
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c = static_cast<int>(blockIdx.x);
  const int nchunk = static_cast<int>((n + kFmCH - 1) / kFmCH);
  const bool last = c == nchunk - 1;
  const long long base = static_cast<long long>(c) * kFmCH;
  // a full chunk (not the call's last): the staging, pairs and stores without per-sample tests
  const bool fast = !last;
  FmPairs p;
  const int e = t * kFmC;
  uint64_t q;
  if (fast) {
    (void)fm_stage<true>(x, n, base, xs);
    q = fm_pairs<true>(kf, xs + e + (e >> 4), kFmC, p);
  } else {
    const int valid = fm_stage(x, n, base, xs);
    q = fm_pairs(kf, xs + e + (e >> 4), valid, p);
  }
  uint64_t agg;
  const uint64_t before = wg_scan_u64(q, tot, agg);
  if (w == 0) {
    uint32_t* my = rec + static_cast<long long>(c) * 8;
    if (!last) {
      if (lane == 0) fm_st64(my, agg);
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the sum is visible before its flag
      if (lane == 0) fm_st(my + 6, epoch);
    }
    uint64_t excl = 0;
    // lane l reads the records of chunks b - L l - j, j < L: 64 L predecessors per step,
    // their flag loads all issued before any is tested
    constexpr int L = kFmLb;
    for (int b = c - 1;; b -= 64 * L) {
      // every flag load of the step issued at once (clamped index; no short-circuit
      // that would serialise them), then every value load
      uint32_t f6[L], f7[L];
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const int k = max(b - L * lane - j, 0);
        f6[j] = fm_ld(rec + static_cast<long long>(k) * 8 + 6);
        f7[j] = fm_ld(rec + static_cast<long long>(k) * 8 + 7);
      }
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const int k = b - L * lane - j;
        if (k >= 0 && f6[j] != epoch && f7[j] != epoch) {  // not yet published: bounded wait
          const uint32_t* pr = rec + static_cast<long long>(k) * 8;
          bool seen = false;  // (spin 0: time out at once, test-only)
          for (uint32_t it = 0; it < spin && !seen; ++it) {
            __builtin_amdgcn_s_sleep(2);
            f7[j] = fm_ld(pr + 7);
            f6[j] = fm_ld(pr + 6);
            seen = f7[j] == epoch || f6[j] == epoch;
          }
          if (!seen) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
      uint64_t vv[L];
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const int k = max(b - L * lane - j, 0);
        vv[j] = fm_ld64(rec + static_cast<long long>(k) * 8 + (f7[j] == epoch ? 2 : 0));
      }
      uint64_t all = 0, upto = 0;  // the lane's L terms; its terms up to its nearest closing one
      int mine = L;                // the lane's nearest closing record (L: none)
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const int k = b - L * lane - j;
        const bool closes = k < 0 || f7[j] == epoch;
        const uint64_t v = k >= 0 ? vv[j] : (k == -1 ? carry_in[0] : 0);  // the carried phase before chunk 0
        all += v;
        if (mine == L) {
          upto += v;
          if (closes) mine = j;
        }
      }
      const unsigned long long bal = __ballot(mine < L);
      const int first = bal ? __builtin_ctzll(bal) : 64;  // the lane holding the nearest closing record
      uint64_t term = lane < first ? all : (lane == first ? upto : 0);
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t lo = __shfl_xor(static_cast<uint32_t>(term), off, 64);
        const uint32_t hi = __shfl_xor(static_cast<uint32_t>(term >> 32), off, 64);
        term += (static_cast<uint64_t>(hi) << 32) | lo;
      }
      excl += term;
      if (first < 64) break;
    }
    if (lane == 0) {
      if (!last) {
        fm_st64(my + 2, excl + agg);
        __builtin_amdgcn_s_waitcnt(0x0F70);
        fm_st(my + 7, epoch);
      } else {
        carry_out[0] = excl + agg;  // the carried phase of the next call (exact mod 2 pi)
      }
      excl_sh = excl;
    }
  }
  __syncthreads();
  if (fast) fm_out<true>(p, excl_sh + before, gain, o, k0, ys, y, base, n);
  else fm_out(p, excl_sh + before, gain, o, k0, ys, y, base, n);
}

}  // namespace

void launch_am_mod(const float* x, f2* y, long long n, uint64_t k0, const OscDev& o, float cl, float mi, float g,
                   bool clamp, hipStream_t s) {
  if (n <= 0) return;
  k_am_mod<<<grid_for(n), NT, 0, s>>>(x, y, n, k0, o, cl, mi, g, clamp ? 1 : 0);
  ORION_LAUNCH_CHECK();
}

void launch_ssb_mod_front(const float* x, float* u, long long n, uint64_t k0, const OscDev& o, hipStream_t s) {
  if (n <= 0) return;
  k_ssb_mod_front<<<grid_for(n), NT, 0, s>>>(x, u, n, k0, o);
  ORION_LAUNCH_CHECK();
}

void launch_pm_mod(const float* x, f2* y, long long n, uint64_t k0, const OscDev& o, float kp, float g, hipStream_t s) {
  if (n <= 0) return;
  k_pm_mod<<<grid_for(n), NT, 0, s>>>(x, y, n, k0, o, kp, g);
  ORION_LAUNCH_CHECK();
}

void launch_ssb_mod_back(const float* v, f2* y, long long n, uint64_t k0, const OscDev& o, float side, hipStream_t s) {
  if (n <= 0) return;
  k_ssb_mod_back<<<grid_for(n), NT, 0, s>>>(v, y, n, k0, o, side);
  ORION_LAUNCH_CHECK();
}

long long fm_mod_chunks(long long n) { return (n + kFmCH - 1) / kFmCH; }

void launch_fm_mod_sp(const float* x, f2* y, long long n, float kf, float gain, uint32_t* rec, uint32_t epoch,
                      const uint64_t* carry_in, uint64_t* carry_out, uint64_t k0, const OscDev& o, int* err,
                      hipStream_t s) {
  if (n <= 0) return;
  const long long nchunk = fm_mod_chunks(n);
  if (nchunk > (1LL << 30)) throw HipError("FM modulator: input too long");
  k_fm_mod_sp<<<static_cast<int>(nchunk), NT, 0, s>>>(x, y, n, kf, gain, rec, epoch, carry_in, carry_out, k0, o, err,
                                                     spin_limit());
  ORION_LAUNCH_CHECK();
}

void launch_fm_mod(const float* x, f2* y, long long n, float kf, float gain, uint64_t* sums,
                   const uint64_t* carry_in, uint64_t* carry_out, uint64_t k0, const OscDev& o, hipStream_t s) {
  if (n <= 0) return;
  const long long nchunk = fm_mod_chunks(n);
  if (nchunk > (1LL << 30)) throw HipError("FM modulator: input too long");
  const int g = static_cast<int>(nchunk);
  k_fm_mod_sum<<<g, NT, 0, s>>>(x, n, kf, sums);
  k_fm_mod_carry<<<1, NT, 0, s>>>(sums, g, carry_in, carry_out);
  k_fm_mod_apply<<<g, NT, 0, s>>>(x, y, n, kf, gain, sums, k0, o);
  ORION_LAUNCH_CHECK();
}

}  // namespace orion
