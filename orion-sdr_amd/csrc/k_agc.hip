// k_agc.hip — AgcRms / AgcRmsIq (dsp/agc.rs:7-150) and CwKeyedMod (modulate/cw.rs:9-87)
// on the device: both are the same switched one-pole envelope recurrence.
//
// The reference's envelope is a data-dependent recurrence
//   env <- a(x2 > env) * env + (1 - a) * x2,  a in {attack_a, release_a}
// (agc.rs:33-41). In real arithmetic it is a continuous piecewise-linear map of
// env with slopes <= amax = max(attack_a, release_a), so two trajectories over the
// same input approach each other by amax per sample. Pass 1 (k_agc) exploits
// that: each lane owns a chunk of L samples, starts W samples early (amax^W <
// 1e-9, an envelope-only walk) from the reference's seed rule applied there, and
// records the envelope it entered its chunk with (ent[c]) and the one it left
// with (ext[c]).
//
// In f32 the contraction is NOT guaranteed: near a constant x2 with a close to 1
// the rounded map has a band of exact fixed points about ulp/(1-a) wide, and a
// warm-up trajectory can settle on a different fixed point than the sequential
// one. So exactness is proved, not assumed: chunk c's outputs are the sequential
// ones iff its entering envelope equals chunk c-1's true exit (by induction from
// chunk 0, which starts from the carried state). k_agc_check finds the first
// chunk whose ent differs (bitwise) from its predecessor's ext; k_agc_fix (one
// wave) re-runs from there, one chunk after another from the true exit, until a
// chunk's recorded entry agrees again, then searches for the next disagreement.
// Every output is therefore the reference's sequential f32 result. Typical
// signals need no re-run; a long constant stretch (the ADVICE case) degrades to an
// in-order walk of the stretch (agc_wave_walk), never to a
// wrong answer.
//
// Per sample: the reference's f32 ops in its order, no FMA contraction
// (-ffp-contract=off), correctly rounded sqrt and divide.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "blocks.hpp"
#include "hip_common.hpp"
#include "osc.hpp"

namespace orion {
namespace {

struct AgcK {
  float att, rel, tgt, gmin, gmax;
};

// The switched one-pole envelope, env <- a * env + (1 - a) * d with a = att when
// up(d, env) else rel, as a policy over the per-sample ops (the walks and the
// exactness machinery below are shared):
//   AgcPol<IQ> — dsp/agc.rs:33-75 / :124-150: d = |x|^2, up = d > env, seed env = max(d0,
//     1e-12) when the carried env is 0 (agc.rs:57-60), out = clamp(tgt / max(sqrt(env),
//     1e-6), gmin, gmax) * x.
//   CwPol — modulate/cw.rs:45-87 CwKeyedMod: d = clamp(x, 0, 1), up = d >= env, no
//     reseed, out = mix_with_nco((env * gain, 0), nco) (the non-FMA product, nco.rs:63-66)
//     with the tone Nco's phasor (osc.hpp RefOsc: the reference recurrence, tabulated).
template <bool IQ>
struct AgcPol {
  using In = typename std::conditional<IQ, float2, float>::type;
  using Out = In;
  AgcK k;
  float att, rel, oma, omr;
  __device__ __forceinline__ float drive(In v) const {
    if constexpr (IQ) return v.x * v.x + v.y * v.y;
    else return v * v;
  }
  __device__ __forceinline__ bool up(float d, float env) const { return d > env; }
  __device__ __forceinline__ float seed(float env, float d0) const { return env == 0.0f ? fmaxf(d0, 1e-12f) : env; }
  __device__ __forceinline__ float warm_seed(float d) const { return fmaxf(d, 1e-12f); }
  static constexpr bool kBracket = false;  // the envelope (a power) has no a-priori bound
  static constexpr float kLo = 0.0f, kHi = 0.0f;
  struct Aux {};
  __device__ __forceinline__ Aux aux(long long) const { return {}; }
  __device__ __forceinline__ Out out(In v, float env, Aux) const {
    const float rms = fmaxf(sqrtf(env), 1e-6f);
    const float g = fminf(fmaxf(k.tgt / rms, k.gmin), k.gmax);
    if constexpr (IQ) return make_float2(g * v.x, g * v.y);
    else return g * v;
  }
};
struct CwPol {
  using In = float;
  using Out = float2;
  float att, rel, oma, omr, gain;
  uint64_t k0;  // sample i of the call: oscillator output k0 + i (the Nco, cw.rs:27)
  OscDev osc;
  __device__ __forceinline__ float drive(In v) const { return v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v); }  // f32::clamp
  __device__ __forceinline__ bool up(float d, float env) const { return d >= env; }
  __device__ __forceinline__ float seed(float env, float) const { return env; }
  __device__ __forceinline__ float warm_seed(float d) const { return d; }
  // env stays in [0, 1] (convex combinations of env_0 = 0 and clamped targets; in f32
  // too: a + (1 - a) rounds to 1): a warm-up from both ends brackets the true envelope
  static constexpr bool kBracket = true;
  static constexpr float kLo = 0.0f, kHi = 1.0f;
  // the tone Nco's phasor of sample i (a table read: the walks issue a batch's reads
  // with its inputs, ahead of the envelope chain)
  using Aux = f2;
  __device__ __forceinline__ Aux aux(long long i) const { return osc_at(osc, k0 + static_cast<uint64_t>(i)); }
  __device__ __forceinline__ Out out(In, float env, Aux p) const {
    const float m = env * gain;
    return make_float2(m * p.x - 0.0f * p.y, m * p.y + 0.0f * p.x);
  }
};

constexpr int kB = 16;

// Walks samples [s, e) of one lane in batches of kB, the next batch's loads issued
// before the current batch's recurrence. OUT = false: envelope only (the warm-up).
template <class Pol, bool OUT>
__device__ __forceinline__ float agc_walk(const typename Pol::In* __restrict__ x, typename Pol::Out* __restrict__ y,
                                          long long s, long long e, float env, const Pol& P) {
  using T = typename Pol::In;
  using A = typename Pol::Aux;
  T cur[kB], nxt[kB];
  A ca[kB], na[kB];
#pragma unroll
  for (int j = 0; j < kB; ++j) {
    cur[j] = s + j < e ? x[s + j] : T{};
    if constexpr (OUT) ca[j] = s + j < e ? P.aux(s + j) : A{};
  }
  auto walk = [&](auto same) {
    for (long long base = s; base < e; base += kB) {
      const long long nb = base + kB;
#pragma unroll
      for (int j = 0; j < kB; ++j) {
        nxt[j] = nb + j < e ? x[nb + j] : T{};
        if constexpr (OUT) na[j] = nb + j < e ? P.aux(nb + j) : A{};
      }
#pragma unroll
      for (int j = 0; j < kB; ++j) {
        const long long i = base + j;
        const float d = P.drive(cur[j]);
        float ne;
        if constexpr (decltype(same)::value) {
          ne = P.att * env + P.oma * d;  // one coefficient pair (agc_wave_walk_n)
        } else {
          const bool up = P.up(d, env);
          ne = (up ? P.att : P.rel) * env + (up ? P.oma : P.omr) * d;  // agc.rs:40, cw.rs:58-62
        }
        if (i < e) {
          env = ne;
          if constexpr (OUT) y[i] = P.out(cur[j], env, ca[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < kB; ++j) {
        cur[j] = nxt[j];
        if constexpr (OUT) ca[j] = na[j];
      }
    }
  };
  if (P.att == P.rel && P.oma == P.omr) walk(std::true_type{});
  else walk(std::false_type{});
  return env;
}

// Two trajectories over [s, e) (envelope only), from the bracket's ends: once they meet
// they stay equal (the same map), and the maps are monotone in env, so the true envelope,
// which starts between them, meets them too. Returns whether they met by e (the merged
// envelope in lo); exactness is still checked bitwise (k_agc_check).
template <class Pol>
__device__ __forceinline__ bool agc_walk2(const typename Pol::In* __restrict__ x, long long s, long long e, float& lo,
                                          float& hi, const Pol& P) {
  using T = typename Pol::In;
  T cur[kB], nxt[kB];
#pragma unroll
  for (int j = 0; j < kB; ++j) cur[j] = s + j < e ? x[s + j] : T{};
  for (long long base = s; base < e; base += kB) {
    const long long nb = base + kB;
#pragma unroll
    for (int j = 0; j < kB; ++j) nxt[j] = nb + j < e ? x[nb + j] : T{};
    const bool same = P.att == P.rel && P.oma == P.omr;
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      const float d = P.drive(cur[j]);
      const bool ul = same || P.up(d, lo), uh = same || P.up(d, hi);
      const float nl = (ul ? P.att : P.rel) * lo + (ul ? P.oma : P.omr) * d;
      const float nh = (uh ? P.att : P.rel) * hi + (uh ? P.oma : P.omr) * d;
      if (base + j < e) {
        lo = nl;
        hi = nh;
      }
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) cur[j] = nxt[j];
    if (__float_as_uint(lo) == __float_as_uint(hi)) {  // met: one trajectory for the rest
      lo = agc_walk<Pol, false>(x, nullptr, nb < e ? nb : e, e, lo, P);
      hi = lo;
      return true;
    }
  }
  return __float_as_uint(lo) == __float_as_uint(hi);
}
constexpr unsigned kNanEnt = 0x7FC00001u, kNanExt = 0x7FC00002u;  // unknown entry / exit: never equal

// One wave walks samples [s, e) in order (the re-runs of k_agc_fix and k_agc_fix_runs,
// the sequential path and the wave-per-chunk pass 1). The 64 lanes load 64 samples
// (coalesced, the next 64 in flight) and form d and both candidate (1 - a) * d products
// into LDS (sm: 4 x 64 floats of this wave); then every lane runs the envelope chain over
// the 64 values read back as broadcast b128 reads, 16 at a time (compare, two selects,
// one multiply, one add per sample: the reference's f32 ops and order), lane 0 records
// every step's envelope in LDS (four b128 writes per 16 steps), and each lane then reads
// its own sample's envelope back and forms its output. NT trajectories (1, or 2 for a
// bracketed warm-up: from env[0] and env[1]) share the broadcast values. When both
// branches use the same coefficients (att == rel and oma == omr: CwKeyedMod with rise ==
// fall) the compare and selects cannot change a bit and the chain is the multiply and
// the add alone. (~27 ns per sample when the chain read its values by v_readlane.)
template <class Pol, bool OUT, int NT>
__device__ __forceinline__ void agc_wave_walk_n(const typename Pol::In* __restrict__ x,
                                                typename Pol::Out* __restrict__ y, long long s, long long e,
                                                float (&env)[NT], const Pol& P, float* __restrict__ sm) {
  using T = typename Pol::In;
  using A = typename Pol::Aux;
  const int lane = threadIdx.x & 63;
  const bool uni = P.att == P.rel && P.oma == P.omr;  // kernel-argument uniform
  // inputs (and output phasors) of the next kAhead blocks in flight: a block's chain
  // (~64 x 10 cycles) is shorter than a load's latency
  constexpr int kAhead = 4;
  T q[kAhead];
  A qa[kAhead];
  // (unconditional loads at a clamped index: a conditional one makes the compiler's wait
  // counting drain every load in flight at its first use)
#pragma unroll
  for (int u = 0; u < kAhead; ++u) {
    const long long i = s + 64 * u + lane;
    q[u] = x[i < e ? i : e - 1];
    if constexpr (OUT) qa[u] = P.aux(i < e ? i : e - 1);
  }
  for (long long base = s; base < e; base += 64) {
    const long long i = base + lane;
    const T cur = q[0];
    A ca{};
    if constexpr (OUT) ca = qa[0];
#pragma unroll
    for (int u = 0; u + 1 < kAhead; ++u) {
      q[u] = q[u + 1];
      if constexpr (OUT) qa[u] = qa[u + 1];
    }
    {
      const long long ip = i + 64 * kAhead;
      q[kAhead - 1] = x[ip < e ? ip : e - 1];
      if constexpr (OUT) qa[kAhead - 1] = P.aux(ip < e ? ip : e - 1);
    }
    const float d = P.drive(cur);
    asm volatile("" ::: "memory");  // the previous block's broadcast reads precede these writes (one wave: DS in order)
    sm[lane] = d;
    sm[64 + lane] = P.oma * d;
    sm[128 + lane] = P.omr * d;
    asm volatile("" ::: "memory");
    const int cnt = e - base < 64 ? static_cast<int>(e - base) : 64;
    auto chain = [&](auto full, auto same) {
      constexpr bool kSame = decltype(same)::value;
      float a64[64];  // one coefficient pair: the block's 64 (1 - a) d values read at once
      if constexpr (kSame) {
#pragma unroll
        for (int t = 0; t < 64; t += 4) {
          const float4 v = *reinterpret_cast<const float4*>(sm + 64 + t);
          a64[t] = v.x; a64[t + 1] = v.y; a64[t + 2] = v.z; a64[t + 3] = v.w;
        }
      }
#pragma unroll
      for (int g = 0; g < 64; g += 16) {
        float dv[16], av[16], rv[16], rec[16];
        if constexpr (kSame) {
#pragma unroll
          for (int t = 0; t < 16; ++t) av[t] = a64[g + t];
        } else {
#pragma unroll
          for (int t = 0; t < 16; t += 4) {
            const float4 u = *reinterpret_cast<const float4*>(sm + g + t);
            const float4 v = *reinterpret_cast<const float4*>(sm + 64 + g + t);
            const float4 w = *reinterpret_cast<const float4*>(sm + 128 + g + t);
            dv[t] = u.x; dv[t + 1] = u.y; dv[t + 2] = u.z; dv[t + 3] = u.w;
            av[t] = v.x; av[t + 1] = v.y; av[t + 2] = v.z; av[t + 3] = v.w;
            rv[t] = w.x; rv[t + 1] = w.y; rv[t + 2] = w.z; rv[t + 3] = w.w;
          }
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          if (decltype(full)::value || g + j < cnt) {
#pragma unroll
            for (int k = 0; k < NT; ++k) {
              if constexpr (kSame) {
                env[k] = P.att * env[k] + av[j];  // agc.rs:40 / cw.rs:58-62 with one coefficient pair
              } else {
                const bool up = P.up(dv[j], env[k]);
                env[k] = (up ? P.att : P.rel) * env[k] + (up ? av[j] : rv[j]);
              }
            }
          }
          rec[j] = env[0];
        }
        if constexpr (OUT) {
          if (lane == 0) {
#pragma unroll
            for (int t = 0; t < 16; t += 4)
              *reinterpret_cast<float4*>(sm + 192 + g + t) = make_float4(rec[t], rec[t + 1], rec[t + 2], rec[t + 3]);
          }
        }
      }
    };
    if (uni) {
      if (cnt == 64) chain(std::true_type{}, std::true_type{});
      else chain(std::false_type{}, std::true_type{});
    } else {
      if (cnt == 64) chain(std::true_type{}, std::false_type{});
      else chain(std::false_type{}, std::false_type{});
    }
    if constexpr (OUT) {
      asm volatile("" ::: "memory");  // lane 0's records precede the reads (one wave: DS in order)
      const float mine = sm[192 + lane];
      if (i < e) y[i] = P.out(cur, mine, ca);
    }
  }
}
template <class Pol, bool OUT = true>
__device__ __forceinline__ float agc_wave_walk(const typename Pol::In* __restrict__ x,
                                               typename Pol::Out* __restrict__ y, long long s, long long e, float env,
                                               const Pol& P, float* __restrict__ sm) {
  float v[1] = {env};
  agc_wave_walk_n<Pol, OUT, 1>(x, y, s, e, v, P, sm);
  return v[0];
}

// The whole call in order by one wave (warm-ups as long as the call itself).
template <class Pol>
__global__ __launch_bounds__(64) void k_agc_seq(const void* __restrict__ in, void* __restrict__ out, long long n,
                                                Pol P, const float* __restrict__ env_in, float* __restrict__ env_out) {
  __shared__ __attribute__((aligned(16))) float sm[256];
  const auto* x = static_cast<const typename Pol::In*>(in);
  float env = P.seed(env_in[0], P.drive(x[0]));
  env = agc_wave_walk<Pol>(x, static_cast<typename Pol::Out*>(out), 0, n, env, P, sm);
  if (threadIdx.x == 0) env_out[0] = env;
}

// Pass 1: chunk c = [c*L, min(c*L+L, n)), warm-up from max(c*L - W, 0).
template <class Pol>
__global__ __launch_bounds__(256) void k_agc(const void* __restrict__ in, void* __restrict__ out, long long n,
                                             long long L, long long W, Pol P, const float* __restrict__ env_in,
                                             float* __restrict__ env_out, float* __restrict__ ent,
                                             float* __restrict__ ext, long long* __restrict__ first_bad) {
  const auto* x = static_cast<const typename Pol::In*>(in);
  auto* y = static_cast<typename Pol::Out*>(out);
  const long long c = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const long long b = c * L;
  if (b >= n) return;
  if (c == 0) first_bad[0] = (n + L - 1) / L;  // "no disagreement" until k_agc_check says otherwise
  const long long e = b + L < n ? b + L : n;
  // A warm-up that would reach back past the call's first sample starts there, from
  // the carried envelope, exactly as chunk 0 does (such chunks are exact).
  const long long s0 = b - W > 0 ? b - W : 0;
  float env;
  if constexpr (Pol::kBracket) {
    if (s0 == 0) {
      env = agc_walk<Pol, false>(x, y, 0, b, P.seed(env_in[0], P.drive(x[0])), P);
    } else {
      float lo = Pol::kLo, hi = Pol::kHi;
      if (!agc_walk2<Pol>(x, s0, b, lo, hi, P)) {  // undetermined: the run fixer re-walks it
        ent[c] = __uint_as_float(kNanEnt);
        ext[c] = __uint_as_float(kNanExt);
        return;
      }
      env = lo;
    }
  } else {
    env = s0 == 0 ? P.seed(env_in[0], P.drive(x[0])) : P.warm_seed(P.drive(x[s0]));
    env = agc_walk<Pol, false>(x, y, s0, b, env, P);
  }
  ent[c] = env;
  env = agc_walk<Pol, true>(x, y, b, e, env, P);
  ext[c] = env;
  if (e == n) env_out[0] = env;
}

// Pass 1 for few chunks (a lane per chunk would leave the chip idle and walk W
// samples with its own strided loads, ~110 ns per sample): one wave per chunk,
// warm-up and chunk by the wave walk (coalesced, inputs in flight a block ahead).
// Same ent / ext records as k_agc, bracketed warm-ups included.
template <class Pol>
__global__ __launch_bounds__(64) void k_agc_wave(const void* __restrict__ in, void* __restrict__ out, long long n,
                                                 long long L, long long W, Pol P, const float* __restrict__ env_in,
                                                 float* __restrict__ env_out, float* __restrict__ ent,
                                                 float* __restrict__ ext, long long* __restrict__ first_bad) {
  __shared__ __attribute__((aligned(16))) float sm[256];
  const auto* x = static_cast<const typename Pol::In*>(in);
  auto* y = static_cast<typename Pol::Out*>(out);
  const long long c = blockIdx.x;
  const long long b = c * L;
  const bool lead = threadIdx.x == 0;
  if (c == 0 && lead) first_bad[0] = (n + L - 1) / L;
  const long long e = b + L < n ? b + L : n;
  const long long s0 = b - W > 0 ? b - W : 0;
  float env;
  if (Pol::kBracket && s0 > 0) {
    float lh[2] = {Pol::kLo, Pol::kHi};
    // both ends in pieces of 256 samples; once they meet, one trajectory for the rest
    long long p = s0;
    for (; p < b && __float_as_uint(lh[0]) != __float_as_uint(lh[1]); p += 256)
      agc_wave_walk_n<Pol, false, 2>(x, y, p, p + 256 < b ? p + 256 : b, lh, P, sm);
    if (p < b) lh[0] = lh[1] = agc_wave_walk<Pol, false>(x, y, p, b, lh[0], P, sm);
    if (__float_as_uint(lh[0]) != __float_as_uint(lh[1])) {  // undetermined: the run fixer re-walks it
      if (lead) {
        ent[c] = __uint_as_float(kNanEnt);
        ext[c] = __uint_as_float(kNanExt);
      }
      return;
    }
    env = lh[0];
  } else {
    env = s0 == 0 ? P.seed(env_in[0], P.drive(x[0])) : P.warm_seed(P.drive(x[s0]));
    env = agc_wave_walk<Pol, false>(x, y, s0, b, env, P, sm);
  }
  if (lead) ent[c] = env;
  env = agc_wave_walk<Pol, true>(x, y, b, e, env, P, sm);
  if (lead) {
    ext[c] = env;
    if (e == n) env_out[0] = env;
  }
}

// Pass 2: the first chunk whose entering envelope is not (bitwise) its
// predecessor's exit; bad (optional): every such chunk flagged.
__global__ __launch_bounds__(256) void k_agc_check(const float* __restrict__ ent, const float* __restrict__ ext,
                                                   long long chunks, long long* __restrict__ first_bad,
                                                   unsigned char* __restrict__ bad) {
  const long long c = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x + 1;
  if (c >= chunks) return;
  const bool b = __float_as_uint(ent[c]) != __float_as_uint(ext[c - 1]);
  if (bad) bad[c] = b ? 1 : 0;
  if (b) atomicMin(reinterpret_cast<unsigned long long*>(first_bad), static_cast<unsigned long long>(c));
}

__global__ void k_agc_reset_first(long long* first_bad, long long chunks) { first_bad[0] = chunks; }

// Pass 2b, the runs of flagged chunks in parallel (one wave per 64 chunks, each run
// fixed by the wave its first chunk falls in): a run's predecessor is unflagged, so
// its recorded exit is taken as true and the run is re-walked in order from it,
// rewriting its chunks' outputs, ent and ext. A run whose predecessor was in fact
// wrong (its predecessor's own predecessor was fixed to a different exit) is caught by
// the second check, and the sequential pass 3 then re-walks from the first chunk
// whose entry disagrees with its predecessor's true exit: every output is still the
// reference's. (The CW keying of the reference's throughput harness: each key-up
// stretch decays multiplicatively and never merges with a warm-up, so it is one run;
// the single-wave pass 3 alone walked every one of them in order.)
template <class Pol>
__global__ __launch_bounds__(64) void k_agc_fix_runs(const void* __restrict__ in, void* __restrict__ out, long long n,
                                                     long long L, Pol P, float* __restrict__ ent, float* __restrict__ ext,
                                                     const unsigned char* __restrict__ bad, long long chunks,
                                                     const long long* __restrict__ first_bad, float* __restrict__ env_out) {
  __shared__ __attribute__((aligned(16))) float sm[256];
  const long long s = blockIdx.x;  // a wave per candidate run start
  if (first_bad[0] >= chunks || s < 1 || s >= chunks || !bad[s] || bad[s - 1]) return;
  const auto* x = static_cast<const typename Pol::In*>(in);
  auto* y = static_cast<typename Pol::Out*>(out);
  const bool lead = threadIdx.x == 0;
  float ex = ext[s - 1];  // unflagged: no fixer writes it
  long long k = s;
  for (; k < chunks && bad[k]; ++k) {
    const long long b = k * L, e = b + L < n ? b + L : n;
    if (lead) ent[k] = ex;
    ex = agc_wave_walk<Pol>(x, y, b, e, ex, P, sm);
    if (lead) ext[k] = ex;
  }
  if (k == chunks && lead) env_out[0] = ex;
}

// Pass 3 (one wave): re-run disagreeing chunks in order from the true exit of
// their predecessor. Exits immediately when pass 2 found nothing.
template <class Pol>
__global__ __launch_bounds__(64) void k_agc_fix(const void* __restrict__ in, void* __restrict__ out, long long n,
                                                long long L, Pol P, const float* __restrict__ ent,
                                                const float* __restrict__ ext, const long long* __restrict__ first_bad,
                                                float* __restrict__ env_out) {
  __shared__ __attribute__((aligned(16))) float sm[256];
  const auto* x = static_cast<const typename Pol::In*>(in);
  auto* y = static_cast<typename Pol::Out*>(out);
  const long long chunks = (n + L - 1) / L;
  long long c = first_bad[0];
  if (c >= chunks) return;
  const int lane = threadIdx.x;
  float ex = ext[c - 1];  // chunks < c are consistent, so this exit is the sequential one
  while (c < chunks) {
    // chunk c entered with the wrong envelope: re-run it from ex, in order
    const long long b = c * L, e = b + L < n ? b + L : n;
    ex = agc_wave_walk<Pol>(x, y, b, e, ex, P, sm);
    ++c;
    // the next chunk whose recorded entry is not the true exit of its predecessor
    long long nxt = chunks;
    for (long long base = c; base < chunks; base += 64) {
      const long long i = base + lane;
      bool bad = false;
      if (i < chunks) {
        const float pred = i == c ? ex : ext[i - 1];
        bad = __float_as_uint(ent[i]) != __float_as_uint(pred);
      }
      const unsigned long long m = __ballot(bad);
      if (m) {
        nxt = base + __ffsll(static_cast<long long>(m)) - 1;
        break;
      }
    }
    if (nxt >= chunks) {
      if (lane == 0) env_out[0] = c == chunks ? ex : ext[chunks - 1];
      return;
    }
    if (nxt != c) ex = ext[nxt - 1];
    c = nxt;
  }
  if (lane == 0) env_out[0] = ex;
}

// Host driver of the three passes for one policy. Chunk length: the extra warm-up
// work per chunk is W/L of a chunk, so L >= W/16 caps the total work at 17 x n; the
// floor keeps >> 1024 waves busy for short warm-ups. W >= n/4: one wave walks the
// call in order (k_agc_seq, ~27 ns per sample, faster than lanes whose own walks are
// that long).
class EnvelopeRunner {
 public:
  explicit EnvelopeRunner(double amax) {
    // amax^W < 1e-9; amax == 1 (or NaN) never forgets: one sequential lane.
    warm_ = amax < 1.0 ? static_cast<long long>(std::ceil(std::log(1e-9) / std::log(amax))) : -1;
    env_.resize(2 * sizeof(float));
    env_.zero();
  }
  long long warm() const { return warm_; }
  long long chunk_len(long long n) const {
    if (warm_ < 0 || warm_ >= n / 4) return n;
    return std::max(256LL, (warm_ + 15) / 16);
  }
  template <class Pol>
  void run(const void* in, void* out, long long n, const Pol& P, hipStream_t s) {
    const long long L = chunk_len(n);
    const long long chunks = (n + L - 1) / L;
    float* e = env_.as<float>();
    float* ein = e + cur_;
    float* eout = e + (cur_ ^ 1);
    cur_ ^= 1;
    if (chunks == 1) {  // one wave, in order
      hipLaunchKernelGGL(k_agc_seq<Pol>, dim3(1), dim3(64), 0, s, in, out, n, P, ein, eout);
      ORION_HIP(hipGetLastError());
      return;
    }
    const size_t need = static_cast<size_t>(chunks) * (2 * sizeof(float) + 1) + 2 * sizeof(long long);
    if (chunk_state_.size() < need) chunk_state_.resize(need);
    long long* first_bad = chunk_state_.as<long long>();
    float* ent = reinterpret_cast<float*>(first_bad + 2);
    float* ext = ent + chunks;
    unsigned char* bad = reinterpret_cast<unsigned char*>(ext + chunks);
    const unsigned grid = static_cast<unsigned>((chunks + 255) / 256);
    const long long W = warm_ < 0 ? 0 : warm_;
    if (chunks <= kWaveChunks) {
      hipLaunchKernelGGL(k_agc_wave<Pol>, dim3(static_cast<unsigned>(chunks)), dim3(64), 0, s, in, out, n, L, W, P, ein,
                         eout, ent, ext, first_bad);
    } else {
      hipLaunchKernelGGL(k_agc<Pol>, dim3(grid), dim3(256), 0, s, in, out, n, L, W, P, ein, eout, ent, ext, first_bad);
    }
    ORION_HIP(hipGetLastError());
    const dim3 cg(static_cast<unsigned>((chunks - 1 + 255) / 256));
    ORION_HIP(hipMemsetAsync(bad, 0, 1, s));  // chunk 0 is never flagged (it starts from the carried state)
    hipLaunchKernelGGL(k_agc_check, cg, dim3(256), 0, s, ent, ext, chunks, first_bad, bad);
    ORION_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_agc_fix_runs<Pol>, dim3(static_cast<unsigned>(chunks)), dim3(64), 0, s, in, out, n, L, P, ent,
                       ext, bad, chunks, first_bad, eout);
    ORION_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_agc_reset_first, dim3(1), dim3(1), 0, s, first_bad, chunks);
    hipLaunchKernelGGL(k_agc_check, cg, dim3(256), 0, s, ent, ext, chunks, first_bad, nullptr);
    ORION_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_agc_fix<Pol>, dim3(1), dim3(64), 0, s, in, out, n, L, P, ent, ext, first_bad, eout);
    ORION_HIP(hipGetLastError());
  }
  void reset() {
    env_.zero();
    cur_ = 0;
  }

 private:
  // Up to this many chunks (four waves per SIMD), a wave per chunk (k_agc_wave).
  static constexpr long long kWaveChunks = 4096;
  long long warm_ = 0;
  DevBuf env_;          // two floats: the carried envelope, ping-ponged per call
  DevBuf chunk_state_;  // first disagreeing chunk, then ent[chunks], ext[chunks]
  int cur_ = 0;
};

class AgcBlock final : public Block {
 public:
  AgcBlock(bool iq, float fs, float attack_ms, float release_ms, float target_rms)
      : iq_(iq), runner_(amax_of(fs, attack_ms, release_ms)) {
    // agc.rs:21 / :97: a(ms) = exp(-1 / (fs * (max(ms, 1e-3) / 1000)))
    k_.att = coef(fs, attack_ms);
    k_.rel = coef(fs, release_ms);
    k_.tgt = std::max(target_rms, 1e-6f);
    k_.gmin = 0.05f;
    k_.gmax = 20.0f;
  }
  const char* name() const override { return iq_ ? "AgcRmsIq" : "AgcRms"; }
  Dt in_type() const override { return iq_ ? Dt::C32 : Dt::F32; }
  Dt out_type() const override { return iq_ ? Dt::C32 : Dt::F32; }
  size_t chunk_quantum() const override { return 1; }  // outputs are the sequential recurrence's, bit for bit
  bool alias_ok() const override { return true; }  // overlapping in/out: staged through a copy
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const long long n = static_cast<long long>(std::min(n_in, out_cap));  // agc.rs:49
    if (n == 0) return {0, 0};
    const size_t bytes = static_cast<size_t>(n) * (iq_ ? 8 : 4);
    const char* ib = static_cast<const char*>(in);
    char* ob = static_cast<char*>(out);
    if (ib < ob + bytes && ob < ib + bytes) {
      // the warm-ups and re-runs read inputs other lanes overwrite: work from a copy
      copy_.resize(std::max(copy_.size(), bytes));
      ORION_HIP(hipMemcpyAsync(copy_.as<void>(), in, bytes, hipMemcpyDeviceToDevice, s));
      in = copy_.as<void>();
    }
    const float oma = 1.0f - k_.att, omr = 1.0f - k_.rel;  // (1 - a) as agc.rs:40 forms it
    if (iq_) runner_.run(in, out, n, AgcPol<true>{k_, k_.att, k_.rel, oma, omr}, s);
    else runner_.run(in, out, n, AgcPol<false>{k_, k_.att, k_.rel, oma, omr}, s);
    return {static_cast<size_t>(n), static_cast<size_t>(n)};
  }
  void reset() override { runner_.reset(); }
  std::vector<float> taps(int which) const override {
    if (which == 1) return {static_cast<float>(runner_.chunk_len(1LL << 24))};
    return {k_.att, k_.rel, k_.tgt, static_cast<float>(runner_.warm())};
  }

 private:
  static float coef(float fs, float ms) { return std::exp(-1.0f / (fs * (std::max(ms, 1e-3f) / 1000.0f))); }
  static double amax_of(float fs, float a, float r) { return std::max(coef(fs, a), coef(fs, r)); }
  bool iq_;
  AgcK k_{};
  EnvelopeRunner runner_;
  DevBuf copy_;  // input copy for overlapping in/out
};

// modulate/cw.rs:9-87 CwKeyedMod: keying envelope f32 -> cf32 IQ.
class CwModBlock final : public Block {
 public:
  CwModBlock(float fs, float tone_hz, float rise_ms, float fall_ms)
      : osc_(tone_hz, fs), runner_(std::max(alpha(fs, rise_ms), alpha(fs, fall_ms))) {
    rise_ = alpha(fs, rise_ms);
    fall_ = alpha(fs, fall_ms);
  }
  const char* name() const override { return "CwKeyedMod"; }
  Dt in_type() const override { return Dt::F32; }
  Dt out_type() const override { return Dt::C32; }
  size_t chunk_quantum() const override { return 1; }  // outputs are the sequential recurrence's, bit for bit
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const long long n = static_cast<long long>(std::min(n_in, out_cap));  // cw.rs:47
    if (n == 0) return {0, 0};
    runner_.run(in, out, n, CwPol{rise_, fall_, 1.0f - rise_, 1.0f - fall_, g_, osc_.count(), osc_.dev(n, s)}, s);
    osc_.advance(static_cast<uint64_t>(n));
    return {static_cast<size_t>(n), static_cast<size_t>(n)};
  }
  void reset() override {
    runner_.reset();
    osc_.reset();
  }
  void set_gain(float g) { g_ = g; }  // cw.rs:39-41
  int configure(int option, long long value) override {
    if (option != kOptNcoTable) return -4;
    if (value < 0 || static_cast<unsigned long long>(value) > kNcoTableMax) return -3;
    osc_.set_budget(static_cast<uint64_t>(value));
    return 0;
  }
  std::vector<float> taps(int) const override { return {rise_, fall_, osc_.osc().w_re, osc_.osc().w_im}; }

 private:
  // cw.rs:27-30: tau = (max(ms, 0.1) * 1e-3) * fs; alpha = exp(-1 / tau)
  static float alpha(float fs, float ms) { return std::exp(-1.0f / ((std::max(ms, 0.1f) * 1e-3f) * fs)); }
  RefOsc osc_;
  EnvelopeRunner runner_;
  float rise_ = 0, fall_ = 0, g_ = 1.0f;
};

}  // namespace

std::unique_ptr<Block> make_agc(bool iq, float fs, float attack_ms, float release_ms, float target_rms) {
  return std::make_unique<AgcBlock>(iq, fs, attack_ms, release_ms, target_rms);
}
std::unique_ptr<Block> make_cw_mod(float fs, float tone_hz, float rise_ms, float fall_ms) {
  return std::make_unique<CwModBlock>(fs, tone_hz, rise_ms, fall_ms);
}
int cw_mod_set_gain(Block* b, float g) {
  auto* c = dynamic_cast<CwModBlock*>(b);
  if (!c) return -4;
  c->set_gain(g);
  return 0;
}

}  // namespace orion
