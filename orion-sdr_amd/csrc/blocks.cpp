// blocks.cpp — Block implementations over the gfx950 kernels (host side).
#include "blocks.hpp"

#include "osc.hpp"
#include "scan_blocks.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

namespace orion {

// ------------------------------------------------------------------ DevBuf --
DevBuf::~DevBuf() {
  if (p_) (void)hipFree(p_);
}
void DevBuf::resize(size_t bytes) {
  if (bytes <= n_) return;
  if (p_) ORION_HIP(hipFree(p_));
  p_ = nullptr;
  n_ = 0;
  ORION_HIP(hipMalloc(&p_, bytes < 256 ? 256 : bytes));
  n_ = bytes < 256 ? 256 : bytes;
}
void DevBuf::zero(hipStream_t s) {
  if (p_) ORION_HIP(hipMemsetAsync(p_, 0, n_, s));
}
void DevBuf::upload(const void* h, size_t bytes, hipStream_t s) {
  resize(bytes);
  ORION_HIP(hipMemcpyAsync(p_, h, bytes, hipMemcpyHostToDevice, s));
  ORION_HIP(hipStreamSynchronize(s));
}

// ------------------------------------------------------------------- Block --
hipStream_t Block::host_stream() {
  if (!hs_) ORION_HIP(hipStreamCreateWithFlags(&hs_, hipStreamNonBlocking));
  return hs_;
}
int* Block::dev_err() {
  if (!err_) {
    void* p = nullptr;
    ORION_HIP(hipHostMalloc(&p, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
    err_ = static_cast<int*>(p);
    __atomic_store_n(err_, 0, __ATOMIC_RELAXED);
  }
  return err_;
}
void Block::check_device_errors() {
  if (err_ && __atomic_exchange_n(err_, 0, __ATOMIC_ACQ_REL) != 0)
    throw HipError(std::string(name()) +
                   ": a cross-workgroup wait of an earlier kernel of this handle timed out; its output is invalid");
}

namespace {
uint32_t g_spin = kSpinDefault;
}
uint32_t spin_limit() { return __atomic_load_n(&g_spin, __ATOMIC_RELAXED); }
void set_spin_limit(uint32_t polls) { __atomic_store_n(&g_spin, polls, __ATOMIC_RELAXED); }

namespace {
std::mutex g_occ_mu;
std::map<std::tuple<const void*, int, int>, int> g_occ;  // (kernel, threads, device) -> per CU
std::map<int, int> g_cus;                                 // device -> CUs
}  // namespace
int resident_per_cu(const void* kernel, int threads) {
  int dev = 0;
  ORION_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(g_occ_mu);
  const auto key = std::make_tuple(kernel, threads, dev);
  auto it = g_occ.find(key);
  if (it != g_occ.end()) return it->second;
  int per_cu = 0;
  ORION_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0));
  per_cu = std::max(1, per_cu);
  g_occ.emplace(key, per_cu);
  return per_cu;
}
int device_cus() {
  int dev = 0;
  ORION_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(g_occ_mu);
  auto it = g_cus.find(dev);
  if (it != g_cus.end()) return it->second;
  int ncu = 0;
  ORION_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  ncu = std::max(1, ncu);
  g_cus.emplace(dev, ncu);
  return ncu;
}

// ---------------------------------------------------------- host path ----
constexpr size_t kPinBytes = 8u << 20;        // one pinned staging buffer at most (two per direction)
constexpr size_t kPipeSamples = 1u << 20;     // calls of >= 2 kPipeSamples take the chunked pipeline
constexpr size_t kDirectBytes = 1u << 20;     // pageable copies up to this size go straight to hipMemcpy

// Parallel memcpy for the pageable staging copies (pageable <-> pinned): one process-wide
// pool of host threads; a copy is cut into >= 1 MiB pieces that the workers and the
// caller take in turn. One thread copies ~20 GB/s, a third of the H2D link (VERDICT r4
// weak 4); a few in parallel keep the copy ahead of the DMA.
class CopyPool {
 public:
  static CopyPool& get() {
    static CopyPool p;
    return p;
  }
  void copy(void* dst, const void* src, size_t bytes) {
    constexpr size_t kPiece = 1u << 20;
    if (bytes < 2 * kPiece || th_.empty()) {
      std::memcpy(dst, src, bytes);
      return;
    }
    std::lock_guard<std::mutex> one(job_mu_);  // one job at a time
    {
      std::lock_guard<std::mutex> g(mu_);
      dst_ = static_cast<char*>(dst);
      src_ = static_cast<const char*>(src);
      bytes_ = bytes;
      pieces_ = std::min<size_t>((bytes + kPiece - 1) / kPiece, 4 * (th_.size() + 1));
      next_.store(0);
      done_.store(0);
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return done_.load() == pieces_; });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }

 private:
  CopyPool() {
    const unsigned hw = std::thread::hardware_concurrency();
    const unsigned n = std::min(7u, hw > 2 ? hw / 2 - 1 : 0u);  // workers besides the caller
    for (unsigned i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  void work() {  // take pieces until none is left
    for (;;) {
      const size_t i = next_.fetch_add(1);
      if (i >= pieces_) return;
      // ceiling division before the 64-B round-up: the pieces always cover bytes_
      // (a floor here dropped the last few bytes when bytes_ % pieces_ != 0)
      const size_t per = ((bytes_ + pieces_ - 1) / pieces_ + 63) & ~size_t(63);
      const size_t off = std::min(bytes_, i * per), len = std::min(per, bytes_ - off);
      std::memcpy(dst_ + off, src_ + off, len);
      if (done_.fetch_add(1) + 1 == pieces_) {
        std::lock_guard<std::mutex> g(mu_);
        done_cv_.notify_all();
      }
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_, job_mu_;
  std::condition_variable cv_, done_cv_;
  char* dst_ = nullptr;
  const char* src_ = nullptr;
  size_t bytes_ = 0, pieces_ = 0;
  std::atomic<size_t> next_{0}, done_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};
void par_copy(void* dst, const void* src, size_t bytes) { CopyPool::get().copy(dst, src, bytes); }

// Created on a handle's first call that needs it (pageable memory above kDirectBytes, or
// the chunked pipeline); the pinned buffers are sized to the calls (kPinBytes at most).
struct Block::HostPipe {
  hipStream_t s_in = nullptr, s_out = nullptr;
  void* pin_in[2] = {nullptr, nullptr};
  void* pin_out[2] = {nullptr, nullptr};
  size_t pin_bytes = 0;
  hipEvent_t ev_in[2] = {nullptr, nullptr}, ev_out[2] = {nullptr, nullptr}, ev_k[2] = {nullptr, nullptr};
  DevBuf din[2], dout[2];
  HostPipe() {
    ORION_HIP(hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking));
    ORION_HIP(hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking));
    for (int b = 0; b < 2; ++b) {
      ORION_HIP(hipEventCreateWithFlags(&ev_in[b], hipEventDisableTiming));
      ORION_HIP(hipEventCreateWithFlags(&ev_out[b], hipEventDisableTiming));
      ORION_HIP(hipEventCreateWithFlags(&ev_k[b], hipEventDisableTiming));
    }
  }
  ~HostPipe() {
    free_pins();
    for (int b = 0; b < 2; ++b) {
      if (ev_in[b]) (void)hipEventDestroy(ev_in[b]);
      if (ev_out[b]) (void)hipEventDestroy(ev_out[b]);
      if (ev_k[b]) (void)hipEventDestroy(ev_k[b]);
    }
    if (s_in) (void)hipStreamDestroy(s_in);
    if (s_out) (void)hipStreamDestroy(s_out);
  }
  void free_pins() {
    for (int b = 0; b < 2; ++b) {
      if (pin_in[b]) (void)hipHostFree(pin_in[b]);
      if (pin_out[b]) (void)hipHostFree(pin_out[b]);
      pin_in[b] = pin_out[b] = nullptr;
    }
    pin_bytes = 0;
  }
  // Grows the pinned buffers. A DMA of this pipe may still be queued (process_host's
  // d2h_staged runs after h2d_staged without a sync), so every copy that
  // reads or writes the old buffers is waited for before they are freed.
  void pins(size_t bytes) {
    bytes = std::min(kPinBytes, (bytes + 4095) & ~size_t(4095));
    if (bytes <= pin_bytes) return;
    for (int b = 0; b < 2; ++b) {
      ORION_HIP(hipEventSynchronize(ev_in[b]));
      ORION_HIP(hipEventSynchronize(ev_out[b]));
    }
    free_pins();
    for (int b = 0; b < 2; ++b) {
      ORION_HIP(hipHostMalloc(&pin_in[b], bytes, hipHostMallocDefault));
      ORION_HIP(hipHostMalloc(&pin_out[b], bytes, hipHostMallocDefault));
    }
    pin_bytes = bytes;
  }
  // host -> device on stream s through the two pinned buffers: the CPU copy of piece
  // c + 1 overlaps the DMA of piece c.
  void h2d_staged(void* dst, const void* src, size_t bytes, hipStream_t s) {
    pins(bytes);
    for (size_t off = 0, c = 0; off < bytes; off += pin_bytes, ++c) {
      const int b = static_cast<int>(c & 1);
      const size_t len = std::min(pin_bytes, bytes - off);
      if (c >= 2) ORION_HIP(hipEventSynchronize(ev_in[b]));  // the DMA of piece c - 2 has read pin_in[b]
      par_copy(pin_in[b], static_cast<const char*>(src) + off, len);
      ORION_HIP(hipMemcpyAsync(static_cast<char*>(dst) + off, pin_in[b], len, hipMemcpyHostToDevice, s));
      ORION_HIP(hipEventRecord(ev_in[b], s));
    }
  }
  // device -> host after everything enqueued on s; synchronous.
  void d2h_staged(void* dst, const void* src, size_t bytes, hipStream_t s) {
    pins(bytes);
    size_t prev_off = 0, prev_len = 0;
    int prev_b = -1;
    for (size_t off = 0, c = 0; off < bytes; off += pin_bytes, ++c) {
      const int b = static_cast<int>(c & 1);
      const size_t len = std::min(pin_bytes, bytes - off);
      ORION_HIP(hipMemcpyAsync(pin_out[b], static_cast<const char*>(src) + off, len, hipMemcpyDeviceToHost, s));
      ORION_HIP(hipEventRecord(ev_out[b], s));
      if (prev_b >= 0) {  // the CPU copy of piece c - 1 overlaps the DMA of piece c
        ORION_HIP(hipEventSynchronize(ev_out[prev_b]));
        par_copy(static_cast<char*>(dst) + prev_off, pin_out[prev_b], prev_len);
      }
      prev_b = b;
      prev_off = off;
      prev_len = len;
    }
    ORION_HIP(hipEventSynchronize(ev_out[prev_b]));
    par_copy(static_cast<char*>(dst) + prev_off, pin_out[prev_b], prev_len);
  }
};

Block::~Block() {
  delete pipe_;
  if (hs_) (void)hipStreamDestroy(hs_);
  if (err_) (void)hipHostFree(err_);
}

Block::HostPipe& Block::pipe() {
  if (!pipe_) pipe_ = new HostPipe();
  return *pipe_;
}

void* host_alloc(size_t bytes) {
  void* p = nullptr;
  ORION_HIP(hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault));
  return p;
}
void host_free(void* p) {
  if (p) ORION_HIP(hipHostFree(p));
}
bool host_is_pinned(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: not an error of ours
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// host -> device / device -> host for process_host: pinned memory by DMA directly,
// small pageable copies by hipMemcpy (HIP stages them), large ones through the pipe.
void Block::h2d(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (!bytes) return;
  if (bytes > kDirectBytes && !host_is_pinned(src)) {
    pipe().h2d_staged(dst, src, bytes, s);
    return;
  }
  ORION_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
}
void Block::d2h(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes > kDirectBytes && !host_is_pinned(dst)) {
    pipe().d2h_staged(dst, src, bytes, s);
    return;
  }
  if (bytes) ORION_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
  ORION_HIP(hipStreamSynchronize(s));
}

WorkReport Block::process_host(const void* in, size_t n_in, void* out, size_t out_cap) {
  hipStream_t s = host_stream();
  const int nch = channels();
  const size_t q = chunk_quantum();
  const size_t ib = dt_size(in_type()), ob = dt_size(out_type());
  // the chunked pipeline needs a quantum whose input and output fit one staging buffer
  // (FirDecimator's 512 m quantum exceeds it for m > 2048)
  if (q && nch == 1 && n_in >= 2 * kPipeSamples && q * std::max(ib, ob) <= kPinBytes)
    return host_chunked(in, n_in, out, out_cap, q);
  stage_in_.resize(std::max<size_t>(1, n_in * nch * ib));
  stage_out_.resize(std::max<size_t>(1, out_cap * nch * ob));
  h2d(stage_in_.as<void>(), in, n_in * nch * ib, s);
  WorkReport w = process_device(stage_in_.as<void>(), n_in, stage_out_.as<void>(), out_cap, s);
  if (nch == 1) {
    d2h(out, stage_out_.as<void>(), w.out_written * ob, s);
  } else {
    if (w.out_written)
      ORION_HIP(hipMemcpy2DAsync(out, out_cap * ob, stage_out_.as<void>(), out_cap * ob, w.out_written * ob, nch,
                                 hipMemcpyDeviceToHost, s));
    ORION_HIP(hipStreamSynchronize(s));
  }
  check_device_errors();
  return w;
}

// Chunks of Q samples (a multiple of q; a chunk's input and output each fit one pinned
// staging buffer) through two device buffer pairs: chunk c's H2D on s_in, its kernel on
// the handle's stream, its D2H on s_out, each waiting on an event of the stage before;
// buffers of parity c & 1 are reused by chunk c + 2 only after its copy-out. The CPU
// copies of pageable memory (into pin_in, out of pin_out) run between the enqueues, so
// they overlap the DMA and the kernels of the neighbouring chunks.
WorkReport Block::host_chunked(const void* in, size_t n_in, void* out, size_t out_cap, size_t q) {
  HostPipe& P = pipe();
  hipStream_t sc = host_stream();
  const size_t ib = dt_size(in_type()), ob = dt_size(out_type());
  const size_t Q = std::max<size_t>(q, kPinBytes / std::max(ib, ob) / q * q);  // Q max(ib, ob) <= kPinBytes
  const size_t n = consumes_all() ? n_in : std::min(n_in, out_cap);  // decim.rs:72-75 / 1:1 min()
  const size_t n_out = std::min(out_len(n), out_cap);
  const bool pin_i = host_is_pinned(in), pin_o = host_is_pinned(out);
  if (!pin_i || !pin_o) P.pins(Q * std::max(ib, ob));
  for (int b = 0; b < 2; ++b) {
    P.din[b].resize(Q * ib);
    P.dout[b].resize(std::max<size_t>(1, out_len(Q)) * ob);
  }
  size_t pend_off[2] = {0, 0}, pend_len[2] = {0, 0};
  bool used[2] = {false, false};
  auto retire = [&](int b) {  // chunk c - 2's copy-out: its buffers of parity b are free after it
    if (!used[b]) return;
    ORION_HIP(hipEventSynchronize(P.ev_out[b]));
    if (pend_len[b] && !pin_o) par_copy(static_cast<char*>(out) + pend_off[b] * ob, P.pin_out[b], pend_len[b] * ob);
    used[b] = false;
  };
  size_t written = 0;
  int c = 0;
  for (size_t off = 0; off < n; off += Q, ++c) {
    const int b = c & 1;
    const size_t len = std::min(Q, n - off);
    retire(b);
    const char* src = static_cast<const char*>(in) + off * ib;
    if (pin_i) {
      ORION_HIP(hipMemcpyAsync(P.din[b].as<void>(), src, len * ib, hipMemcpyHostToDevice, P.s_in));
    } else {
      par_copy(P.pin_in[b], src, len * ib);  // pin_in[b]'s previous DMA (chunk c - 2) is done: retire(b)
      ORION_HIP(hipMemcpyAsync(P.din[b].as<void>(), P.pin_in[b], len * ib, hipMemcpyHostToDevice, P.s_in));
    }
    ORION_HIP(hipEventRecord(P.ev_in[b], P.s_in));
    ORION_HIP(hipStreamWaitEvent(sc, P.ev_in[b], 0));
    const WorkReport w = process_device(P.din[b].as<void>(), len, P.dout[b].as<void>(), out_len(len), sc);
    ORION_HIP(hipEventRecord(P.ev_k[b], sc));
    ORION_HIP(hipStreamWaitEvent(P.s_out, P.ev_k[b], 0));
    const size_t keep = written < n_out ? std::min(w.out_written, n_out - written) : 0;
    if (keep)
      ORION_HIP(hipMemcpyAsync(pin_o ? static_cast<void*>(static_cast<char*>(out) + written * ob) : P.pin_out[b],
                               P.dout[b].as<void>(), keep * ob, hipMemcpyDeviceToHost, P.s_out));
    ORION_HIP(hipEventRecord(P.ev_out[b], P.s_out));
    pend_off[b] = written;
    pend_len[b] = keep;
    used[b] = true;
    written += w.out_written;
  }
  retire(c & 1);  // the older of the two chunks in flight first
  retire((c + 1) & 1);
  ORION_HIP(hipStreamSynchronize(sc));
  check_device_errors();
  return {n, n_out};
}

namespace {

Taps256 taps256(const std::vector<float>& g) {
  Taps256 t{};
  for (size_t i = 0; i < g.size() && i < 256; ++i) t.g[i] = g[i];
  return t;
}

// FirLowpass::dot pairs taps[L-1] with the newest sample and taps[t] with
// x[n-1-t] (dsp/fir.rs:57-66). As a standard FIR y[n] = sum_k g[k] x[n-k]:
// g[0] = taps[L-1], g[k] = taps[k-1].
std::vector<float> fir_lowpass_as_standard(const std::vector<float>& h) {
  std::vector<float> g(h.size());
  g[0] = h.back();
  for (size_t k = 1; k < h.size(); ++k) g[k] = h[k - 1];
  return g;
}

int padded_hist(int K) {
  if (K <= 64) return 64;
  if (K <= 128) return 128;
  if (K <= 256) return 256;
  return K;
}

// ------------------------------------------------------ Rotator / Nco ----
// The oscillator (osc.hpp RefOsc): the reference's own phasor recurrence, tabulated
// at every (re)tune — exact forever when it closes a cycle within the budget, else
// for the budget's outputs, then the drift model; budget 0: the closed form.
class OscBlock : public Block {
 public:
  OscBlock(float f, float fs) : osc_(f, fs) {}
  void reset() override { osc_.reset(); }  // phasor back to 1 + 0j (Rotator::reset_phase, rotator.rs:28-31)
  std::vector<float> taps(int) const override { return {osc_.osc().w_re, osc_.osc().w_im}; }
  void set_freq(float f, float fs) { osc_.retune(f, fs); }
  void seek(uint64_t k) { osc_.seek(k); }  // the phase origin of a time shard (no reference counterpart)
  float fs() const { return osc_.fs(); }
  size_t chunk_quantum() const override { return kRotTile; }  // tiles keep their alignment
  int configure(int option, long long value) override {
    if (option != kOptNcoTable) return -4;
    if (value < 0 || static_cast<unsigned long long>(value) > kNcoTableMax) return -3;
    osc_.set_budget(static_cast<uint64_t>(value));
    return 0;
  }
  // One oscillator pass (launch_osc mode) over n samples, advancing the phase.
  void run(int mode, const void* in, void* out, size_t n, hipStream_t s) {
    launch_osc(mode, static_cast<const f2*>(in), out, static_cast<long long>(n), osc_.count(), osc_.dev(n, s), s);
    osc_.advance(n);
  }

 private:
  RefOsc osc_;
};

// dsp/rotator.rs:8-95: process = rotate_block (cf32 -> cf32); mix_usb_block and
// next / next_cs on the same phasor (osc_mix_usb, osc_next_cs).
class RotatorBlock final : public OscBlock {
 public:
  RotatorBlock(float f, float fs) : OscBlock(f, fs) {}
  const char* name() const override { return "Rotator"; }
  Dt in_type() const override { return Dt::C32; }
  Dt out_type() const override { return Dt::C32; }
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const size_t n = std::min(n_in, out_cap);  // rotator.rs:76
    run(0, in, out, n, s);
    return {n, n};
  }
};

// dsp/nco.rs:11-66: process = mix_with_nco per sample (cf32 -> cf32, the non-FMA
// product); next_cs as a block of phasors (osc_next_cs).
class NcoBlock final : public OscBlock {
 public:
  NcoBlock(float f, float fs) : OscBlock(f, fs) {}
  const char* name() const override { return "Nco"; }
  Dt in_type() const override { return Dt::C32; }
  Dt out_type() const override { return Dt::C32; }
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const size_t n = std::min(n_in, out_cap);
    run(2, in, out, n, s);
    return {n, n};
  }
};

// ------------------------------------------------------ analog modulators --
constexpr float kTauF = 6.28318530717958647692f;  // core::f32::consts::TAU
// ORION_OPT_NCO_TABLE on a block that owns one RefOsc.
int configure_osc(RefOsc& o, int option, long long value) {
  if (option != kOptNcoTable) return -4;
  if (value < 0 || static_cast<unsigned long long>(value) > kNcoTableMax) return -3;
  o.set_budget(static_cast<uint64_t>(value));
  return 0;
}

// modulate/am.rs:9-120 (rf_nco: Rotator, am.rs:28). F32 audio -> C32 IQ.
class AmModBlock final : public Block {
 public:
  AmModBlock(float fs, float rf_hz, float cl, float mi) : osc_(rf_hz, fs), cl_(cl), mi_(mi) {}
  const char* name() const override { return "AmDsbMod"; }
  Dt in_type() const override { return Dt::F32; }
  Dt out_type() const override { return Dt::C32; }
  size_t chunk_quantum() const override { return 4096; }
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const size_t n = std::min(n_in, out_cap);  // am.rs:45
    launch_am_mod(static_cast<const float*>(in), static_cast<f2*>(out), static_cast<long long>(n), osc_.count(),
                  osc_.dev(n, s), cl_, mi_, g_, clamp_, s);
    osc_.advance(n);
    return {n, n};
  }
  void reset() override { osc_.reset(); }
  void set_gain(float g) { g_ = g; }        // am.rs:31-33
  void set_clamp(bool on) { clamp_ = on; }  // am.rs:34-36
  int configure(int option, long long value) override { return configure_osc(osc_, option, value); }
  std::vector<float> taps(int) const override { return {osc_.osc().w_re, osc_.osc().w_im}; }

 private:
  RefOsc osc_;
  float cl_, mi_, g_ = 1.0f;
  bool clamp_ = false;
};

// modulate/pm.rs:9-47 PmDirectPhaseMod (rf_nco: Nco, pm.rs:20). F32 audio -> C32 IQ.
class PmModBlock final : public Block {
 public:
  PmModBlock(float fs, float kp, float rf_hz) : osc_(rf_hz, fs), kp_(kp) {}
  const char* name() const override { return "PmDirectPhaseMod"; }
  Dt in_type() const override { return Dt::F32; }
  Dt out_type() const override { return Dt::C32; }
  size_t chunk_quantum() const override { return 4096; }
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const size_t n = std::min(n_in, out_cap);  // pm.rs:37
    launch_pm_mod(static_cast<const float*>(in), static_cast<f2*>(out), static_cast<long long>(n), osc_.count(),
                  osc_.dev(n, s), kp_, g_, s);
    osc_.advance(n);
    return {n, n};
  }
  void reset() override { osc_.reset(); }
  void set_gain(float g) { g_ = g; }          // pm.rs:24-26
  void set_sensitivity(float kp) { kp_ = kp; }  // pm.rs:27-29
  int configure(int option, long long value) override { return configure_osc(osc_, option, value); }
  std::vector<float> taps(int) const override { return {kp_, osc_.osc().w_re, osc_.osc().w_im}; }

 private:
  RefOsc osc_;
  float kp_, g_ = 1.0f;
};

// modulate/fm.rs:11-74 (rf_nco: Nco, fm.rs:27). F32 audio -> C32 IQ; the running phase
// is carried on the device (a Q0.64 turn count, exact mod 2 pi) so consecutive calls
// chain without a host sync.
class FmModBlock final : public Block {
 public:
  FmModBlock(float fs, float dev_hz, float rf_hz) : fs_(fs), dev_(dev_hz), osc_(rf_hz, fs) {
    for (auto& c : carry_) c.resize(sizeof(uint64_t));
    reset();
  }
  const char* name() const override { return "FmPhaseAccumMod"; }
  Dt in_type() const override { return Dt::F32; }
  Dt out_type() const override { return Dt::C32; }
  size_t chunk_quantum() const override { return 4096; }  // thread groups and chunks keep their alignment
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const size_t n = std::min(n_in, out_cap);  // fm.rs:47
    if (n == 0) return {0, 0};
    const float kf = kTauF * dev_ / fs_;  // fm.rs:48, f32 as in the reference
    const long long nn = static_cast<long long>(n);
    if (single_pass_) {
      const size_t bytes = static_cast<size_t>(fm_mod_chunks(nn)) * 8 * sizeof(uint32_t);
      if (bytes > rec_.size()) {
        rec_.resize(bytes);
        rec_.zero(s);
        epoch_ = 0;
      }
      if (++epoch_ == 0xFFFFFFFFu) {  // never reuse a tag that may sit in a record
        rec_.zero(s);
        epoch_ = 1;
      }
      launch_fm_mod_sp(static_cast<const float*>(in), static_cast<f2*>(out), nn, kf, g_, rec_.as<uint32_t>(), epoch_,
                       carry_[cur_].as<uint64_t>(), carry_[cur_ ^ 1].as<uint64_t>(), osc_.count(), osc_.dev(n, s),
                       dev_err(), s);
    } else {
      sums_.resize(static_cast<size_t>(fm_mod_chunks(nn)) * sizeof(uint64_t));
      launch_fm_mod(static_cast<const float*>(in), static_cast<f2*>(out), nn, kf, g_, sums_.as<uint64_t>(),
                    carry_[cur_].as<uint64_t>(), carry_[cur_ ^ 1].as<uint64_t>(), osc_.count(), osc_.dev(n, s), s);
    }
    cur_ ^= 1;
    osc_.advance(n);
    return {n, n};
  }
  void reset() override {
    for (auto& c : carry_) c.zero();
    ORION_HIP(hipDeviceSynchronize());
    cur_ = 0;
    osc_.reset();
  }
  void set_gain(float g) { g_ = g; }           // fm.rs:37-39
  void set_deviation(float d) { dev_ = d; }    // fm.rs:34-36
  int configure(int option, long long value) override {
    if (option == kOptNcoTable) return configure_osc(osc_, option, value);
    if (option != kOptModPasses) return -4;
    if (value != 0 && value != 1 && value != 3) return -3;
    single_pass_ = value != 3;
    return 0;
  }
  std::vector<float> taps(int) const override { return {kTauF * dev_ / fs_, osc_.osc().w_re, osc_.osc().w_im}; }

 private:
  float fs_, dev_, g_ = 1.0f;
  RefOsc osc_;
  DevBuf carry_[2], sums_, rec_;
  int cur_ = 0;
  uint32_t epoch_ = 0;
  bool single_pass_ = true;  // k_fm_mod_sp, or the three passes (orion_block_configure)
};

// --------------------------------------------------------- FirDecimator ----
class DecimBlock final : public Block {
 public:
  DecimBlock(float fs, size_t m, float cutoff, float trans, int nch) : m_(m < 1 ? 1 : m), nch_(nch) {
    h_ = fir_lowpass_taps(fs, cutoff, trans);  // decim.rs:25-26: FirLowpass::design
    g_ = fir_lowpass_as_standard(h_);
    K_ = static_cast<int>(g_.size());
    // Fast polyphase path (M = 8, Q in {16, 32}) wants taps phase-major.
    if (m_ == 8 && K_ <= 256) {
      const int Q = K_ <= 128 ? 16 : 32;
      std::vector<float> pm(8 * Q, 0.0f);
      for (int k = 0; k < K_; ++k) pm[(k % 8) * Q + k / 8] = g_[k];
      fast_ = taps256(pm);
      hist_len_ = 8 * Q;
    } else {
      hist_len_ = K_;
    }
    g_dev_.upload(g_.data(), g_.size() * sizeof(float));
    for (auto& h : hist_) {
      h.resize(static_cast<size_t>(hist_len_) * nch_ * sizeof(f2));
      h.zero();
    }
    ORION_HIP(hipDeviceSynchronize());
  }
  const char* name() const override { return "FirDecimator"; }
  Dt in_type() const override { return Dt::C32; }
  Dt out_type() const override { return Dt::C32; }
  size_t chunk_quantum() const override { return 512 * m_; }  // the phase restarts at every call: cut at multiples of m
  bool consumes_all() const override { return true; }
  int channels() const override { return nch_; }
  size_t out_len(size_t n) const override { return (n + m_ - 1) / m_; }
  WorkReport process_device(const void* in, size_t n, void* out, size_t out_cap, hipStream_t s) override {
    if (n == 0) return {0, 0};
    const size_t n_write = std::min(out_len(n), out_cap);  // decim.rs:66-67
    const f2* x = static_cast<const f2*>(in);
    launch_decim_batch(x, static_cast<long long>(n), static_cast<long long>(n), hist_[cur_].as<f2>(),
                       hist_len_, static_cast<f2*>(out), static_cast<long long>(out_cap),
                       static_cast<long long>(n_write), nch_, static_cast<int>(m_), K_, fast_,
                       g_dev_.as<float>(), s, hist_[cur_ ^ 1].as<f2>());
    cur_ ^= 1;
    return {n, n_write};  // all input consumed, decim.rs:72-75
  }
  void reset() override {
    for (auto& h : hist_) h.zero();
    ORION_HIP(hipDeviceSynchronize());
  }
  std::vector<float> taps(int) const override { return h_; }

 private:
  size_t m_;
  int nch_;
  std::vector<float> h_, g_;
  int K_ = 0, hist_len_ = 0;
  Taps256 fast_{};
  DevBuf g_dev_, hist_[2];
  int cur_ = 0;
};

// ----------------------------------------------------------- FirLowpass ----
class FirRealBlock final : public Block {
 public:
  FirRealBlock(float fs, float pass, float trans) {
    h_ = fir_lowpass_taps(fs, pass, trans);
    g_ = fir_lowpass_as_standard(h_);
    K_ = static_cast<int>(g_.size());
    hist_len_ = padded_hist(K_);
    std::vector<float> gp(std::max(K_, 256), 0.0f);
    std::copy(g_.begin(), g_.end(), gp.begin());
    fast_ = taps256(gp);
    g_dev_.upload(g_.data(), g_.size() * sizeof(float));
    for (auto& h : hist_) {
      h.resize(hist_len_ * sizeof(float));
      h.zero();
    }
    ORION_HIP(hipDeviceSynchronize());
  }
  const char* name() const override { return "FirLowpass"; }
  Dt in_type() const override { return Dt::F32; }
  Dt out_type() const override { return Dt::F32; }
  size_t chunk_quantum() const override { return 4096; }
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const size_t n = std::min(n_in, out_cap);  // fir.rs:48
    if (n == 0) return {0, 0};
    const float* x = static_cast<const float*>(in);
    launch_fir_real(x, static_cast<long long>(n), hist_[cur_].as<float>(), hist_len_, static_cast<float*>(out),
                    K_, fast_, g_dev_.as<float>(), s, hist_[cur_ ^ 1].as<float>());
    cur_ ^= 1;
    return {n, n};
  }
  void reset() override {
    for (auto& h : hist_) h.zero();
    ORION_HIP(hipDeviceSynchronize());
  }
  std::vector<float> taps(int) const override { return h_; }

 private:
  std::vector<float> h_, g_;
  int K_ = 0, hist_len_ = 0;
  Taps256 fast_{};
  DevBuf g_dev_, hist_[2];
  int cur_ = 0;
};

// --------------------------------------------------------- FirLowpassIq ----
class FirIqBlock final : public Block {
 public:
  // nch > 1: independent channels sharing the taps (one stream per channel, [nch][n]).
  FirIqBlock(std::vector<float> taps, int nch) : h_(std::move(taps)), nch_(nch) {
    if (nch_ < 1) throw std::invalid_argument("FirLowpassIq needs >= 1 channel");
    if (h_.empty()) h_.push_back(1.0f);  // fir.rs:195-197
    K_ = static_cast<int>(h_.size());
    hist_len_ = padded_hist(K_);
    std::vector<float> gp(std::max(K_, 256), 0.0f);
    std::copy(h_.begin(), h_.end(), gp.begin());  // taps[0] <-> newest (fir.rs:233-235)
    fast_ = taps256(gp);
    g_dev_.upload(h_.data(), h_.size() * sizeof(float));
    for (auto& h : hist_) {
      h.resize(static_cast<size_t>(nch_) * hist_len_ * sizeof(f2));
      h.zero();
    }
    zeros_.resize(hist_len_ * sizeof(f2));
    zeros_.zero();
    ORION_HIP(hipDeviceSynchronize());
  }
  const char* name() const override { return "FirLowpassIq"; }
  Dt in_type() const override { return Dt::C32; }
  Dt out_type() const override { return Dt::C32; }
  int channels() const override { return nch_; }
  size_t chunk_quantum() const override { return 4096; }
  WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap, hipStream_t s) override {
    const size_t n = std::min(n_in, out_cap);  // fir.rs:288
    if (n == 0) return {0, 0};
    const f2* x = static_cast<const f2*>(in);
    launch_fir_iq(x, static_cast<long long>(n), hist_[cur_].as<f2>(), hist_len_, static_cast<f2*>(out),
                  static_cast<long long>(n), 0, K_, fast_, g_dev_.as<float>(), s, hist_[cur_ ^ 1].as<f2>(), nch_,
                  static_cast<long long>(n_in), static_cast<long long>(out_cap));
    cur_ ^= 1;
    return {n, n};
  }
  void reset() override {
    for (auto& h : hist_) h.zero();
    ORION_HIP(hipDeviceSynchronize());
  }
  std::vector<float> taps(int) const override { return h_; }
  // fir.rs:260-276: reset, then y[i] = streamed[i + d] over x padded with zeros.
  void aligned(void* io, size_t n, hipStream_t s) {
    if (nch_ != 1) throw std::invalid_argument("filter_aligned: single-channel FirLowpassIq only");
    reset();
    if (n == 0) return;
    const long long d = (K_ - 1) / 2;
    const long long ne = fir_iq_aligned_edges(static_cast<long long>(n), K_);
    if (hist_len_ >= (K_ <= 64 ? 64 : K_ <= 128 ? 128 : 256)) {
      if (edges_.size() < static_cast<size_t>(ne) * sizeof(f2)) edges_.resize(static_cast<size_t>(ne) * sizeof(f2));
      if (launch_fir_iq_aligned_inplace(static_cast<f2*>(io), static_cast<long long>(n), d, K_, fast_, edges_.as<f2>(),
                                        ne, hist_[cur_ ^ 1].as<f2>(), hist_len_, s)) {
        cur_ ^= 1;
        return;
      }
    }
    scratch_.resize(n * sizeof(f2));
    ORION_HIP(hipMemcpyAsync(scratch_.as<void>(), io, n * sizeof(f2), hipMemcpyDeviceToDevice, s));
    launch_fir_iq(scratch_.as<f2>(), static_cast<long long>(n), zeros_.as<f2>(), hist_len_, static_cast<f2*>(io),
                  static_cast<long long>(n), d, K_, fast_, g_dev_.as<float>(), s);
    // The reference leaves the delay line holding the last K samples it pushed
    // (x[n-K+d+1 .. n-1] then d zeros); a following streaming call sees them.
    // Reproduce by rebuilding the history from [x | d zeros].
    tail_.resize((n + d) * sizeof(f2) + 16);
    ORION_HIP(hipMemsetAsync(tail_.as<void>(), 0, (n + d) * sizeof(f2), s));
    ORION_HIP(hipMemcpyAsync(tail_.as<void>(), scratch_.as<void>(), n * sizeof(f2), hipMemcpyDeviceToDevice, s));
    launch_hist_update_c(tail_.as<f2>(), static_cast<long long>(n + d), zeros_.as<f2>(), hist_[cur_ ^ 1].as<f2>(),
                         hist_len_, s);
    cur_ ^= 1;
  }

 private:
  std::vector<float> h_;
  int K_ = 0, hist_len_ = 0;
  Taps256 fast_{};
  DevBuf g_dev_, hist_[2], zeros_, scratch_, tail_, edges_;
  int nch_ = 1;
  int cur_ = 0;
};

// ------------------------------------------------------------ WBFM chain ----
// The reference composition (docs/demodulate.md:128-133) on three engines:
//   kPathSeg   k_wbfm_seg, one kernel (m = 8, <= 128 decimator and audio taps, an
//              LpCascade that forgets within a sub-range: the WBFM defaults);
//   kPathSplit k_wbfm_front2 + k_wbfm_back (same designs, LpCascade warm-up of kBackW);
//   kPathGraph the four blocks themselves, stage by stage through HBM: Rotator (the
//              reference's own recurrence) -> FirDecimator (any m, any taps) ->
//              FmQuadratureDemod (exact scan, any LpCascade) -> FirLowpass (any taps).
//              Any design the reference's constructors accept (decim.rs:24-37,
//              fir.rs:16-44, fm.rs:17-31).
// The fused paths mix with the closed-form phasor of the recurrence's LONG-RUN step
// (design.hpp rec_mean_step): the reference's f32 Rotator drifts from its nominal step
// by ~1e-8 rad per sample (-1.5 MHz / 10 MHz: +1.15e-8), which the discriminator turns
// into a DC offset of ~6e-7 of full-scale audio; the mean step reproduces it, the
// per-step jitter is below the decimator's passband rounding.
class WbfmBlock final : public Block {
 public:
  WbfmBlock(const WbfmParams& p, const std::vector<float>& f_off)
      : p_(p), nch_(static_cast<int>(f_off.size())), f_off_(f_off) {
    if (p.m < 1) throw std::invalid_argument("WBFM chain: decimation m must be >= 1");
    if (nch_ < 1) throw std::invalid_argument("WBFM chain needs >= 1 channel");
    h_dec_ = fir_lowpass_taps(p.fs, p.dec_cutoff, p.dec_trans);
    const float fs2 = p.fs / static_cast<float>(p.m);
    h_aud_ = fir_lowpass_taps(fs2, p.audio_pass, p.audio_trans);
    fused_ok_ = p.m == kWbfmM && h_dec_.size() <= 128 && h_aud_.size() <= 128;
    if (fused_ok_) build_fused(f_off);
    for (int i = 0; i < 2; ++i) {
      carry_[i].resize(static_cast<size_t>(nch_) * kWbfmCarry * sizeof(float));
      hist_[i].resize(static_cast<size_t>(nch_) * kWbfmHist * sizeof(f2));
    }
    reset();
  }
  const char* name() const override { return "WbfmChain"; }
  Dt in_type() const override { return Dt::C32; }
  Dt out_type() const override { return Dt::F32; }
  bool consumes_all() const override { return true; }
  int channels() const override { return nch_; }
  size_t out_len(size_t n) const override { return (n + p_.m - 1) / p_.m; }
  WorkReport process_device(const void* in, size_t n, void* out, size_t out_cap, hipStream_t s) override {
    if (n == 0) return {0, 0};
    const size_t n_dec = std::min(out_len(n), out_cap);
    const int path = resolved_path();
    if (path == kPathGraph) {
      graph(static_cast<const f2*>(in), n, static_cast<float*>(out), out_cap, n_dec, s);
      k0_ += n;
      processed_ = true;
      return {n, n_dec};
    }
    const int nxt = cur_ ^ 1;
    if (n_dec == 0) {  // decimator consumed input, demod saw nothing (core.rs chain semantics)
      const f2* x = static_cast<const f2*>(in);
      launch_hist_update_c(x, static_cast<long long>(n), hist_[cur_].as<f2>(), hist_[nxt].as<f2>(),
                           kWbfmHist, s, nch_, static_cast<long long>(n));
      ORION_HIP(hipMemcpyAsync(carry_[nxt].as<void>(), carry_[cur_].as<void>(), carry_[cur_].size(),
                               hipMemcpyDeviceToDevice, s));
    } else {
      WbfmArgs a{};
      a.x = static_cast<const f2*>(in);
      a.x_stride = static_cast<long long>(n);
      a.n = static_cast<long long>(n);
      a.y = static_cast<float*>(out);
      a.y_stride = static_cast<long long>(out_cap);
      a.n_dec = static_cast<long long>(n_dec);
      a.k0 = static_cast<long long>(k0_);
      a.step = step_.as<uint64_t>();
      a.tab = tab_.as<f2>();
      a.carry_in = carry_[cur_].as<float>();
      a.carry_out = carry_[nxt].as<float>();
      a.hist_in = hist_[cur_].as<f2>();
      a.hist_out = hist_[nxt].as<f2>();
      a.lanemats = lanemats_.as<double>();
      a.afrag = afrag_.as<void>();
      if (path == kPathSeg) {
        const long long slots = wbfm_seg_slots(static_cast<long long>(n_dec), nch_);
        if (static_cast<size_t>(slots) * kSeg4Slot * 4 > hand_.size()) hand_.resize(static_cast<size_t>(slots) * kSeg4Slot * 4);
        if (static_cast<size_t>(slots) * 3 * 4 > flags_.size()) {
          flags_.resize(static_cast<size_t>(slots) * 3 * 4);
          flags_.zero(s);  // epochs start at 1: a zeroed flag never matches
        }
        a.hand = hand_.as<uint32_t>();
        a.flags = flags_.as<uint32_t>();
        a.err = dev_err();
        a.spin = spin_limit();
        a.epoch = ++epoch_;
        static const char* trace_path = std::getenv("ORION_WBFM_TRACE");  // debug only: per-wave phase timestamps
        if (trace_path) {
          trace_.resize(static_cast<size_t>(slots) * kFuTracePoints * 8);
          trace_.zero(s);
          a.trace = trace_.as<long long>();
        }
        if (epoch_ == 0xFFFFFFFFu) {  // never reuse a tag that may sit in a flag
          flags_.zero(s);
          epoch_ = 0;
        }
        launch_wbfm_seg(a, cf_, cs_, nch_, max_seg_, s);
        if (trace_path) {  // debug: dump this launch's timestamps (overwrites: last launch wins)
          std::vector<long long> h(static_cast<size_t>(slots) * kFuTracePoints);
          ORION_HIP(hipMemcpyAsync(h.data(), trace_.as<void>(), h.size() * 8, hipMemcpyDeviceToHost, s));
          ORION_HIP(hipStreamSynchronize(s));
          if (FILE* f = std::fopen(trace_path, "wb")) {
            std::fwrite(h.data(), 8, h.size(), f);
            std::fclose(f);
          }
        }
      } else {
        phi_.resize(static_cast<size_t>(nch_) * n_dec * sizeof(float) + 64);
        a.phi = phi_.as<float>();
        a.phi_stride = static_cast<long long>(n_dec);
        launch_wbfm(a, cf_, cb_, nch_, s);
      }
    }
    cur_ = nxt;
    k0_ += n;
    processed_ = true;
    return {n, n_dec};
  }
  void reset() override {
    std::vector<float> c0(static_cast<size_t>(nch_) * kWbfmCarry, 0.0f);
    for (int ch = 0; ch < nch_; ++ch) c0[ch * kWbfmCarry + 4] = 1.0f;  // prev = 1+0j (fm.rs:29)
    for (int i = 0; i < 2; ++i) {
      carry_[i].upload(c0.data(), c0.size() * sizeof(float));
      hist_[i].zero();
    }
    ORION_HIP(hipDeviceSynchronize());
    cur_ = 0;
    // Every path restarts at the seek origin (0 unless orion_wbfm_chain_seek set one):
    // the graph path's Rotator is re-sought there when its stages are rebuilt.
    k0_ = seek_;
    processed_ = false;
    stages_.clear();  // the graph path's blocks restart from their constructors' state
  }
  std::vector<float> taps(int which) const override { return which == 0 ? h_dec_ : h_aud_; }
  // The graph path's stages are blocks with error words of their own (the FM demod's
  // cross-workgroup scan): a timeout in any of them invalidates the chain's output.
  void check_device_errors() override {
    Block::check_device_errors();
    for (Stages& st : stages_)
      for (Block* b : {st.rot.get(), st.dec.get(), st.fm.get(), st.aud.get()}) {
        try {
          b->check_device_errors();
        } catch (const HipError& e) {
          throw HipError(std::string(name()) + " (graph path stage): " + e.what());
        }
      }
  }
  // Moves the NCO phase origin only; the carried filter state (decimator and FIR
  // history, discriminator sample, LpCascade) is kept on every path, as the fused
  // paths keep their carry.
  // On the fused paths the decimator history is kept as RAW input and re-mixed by each
  // call at its own indices (phasor e^{j k step}); a mid-stream seek therefore rotates it
  // by e^{j (k_old - k_new) step}, so that it re-mixes to the samples it was mixed to
  // before: what the graph path's decimator (which holds mixed samples) keeps.
  void seek(uint64_t index) {
    if (processed_ && fused_ok_ && resolved_path() != kPathGraph && index != k0_) rebase_history(index);
    k0_ = index;
    seek_ = index;
    for (Stages& st : stages_) osc_seek(st.rot.get(), index);
  }
  void rebase_history(uint64_t index) {
    std::vector<f2> h(static_cast<size_t>(nch_) * kWbfmHist);
    ORION_HIP(hipDeviceSynchronize());  // the last call has written hist_[cur_]
    ORION_HIP(hipMemcpy(h.data(), hist_[cur_].as<void>(), h.size() * sizeof(f2), hipMemcpyDeviceToHost));
    for (int ch = 0; ch < nch_; ++ch) {
      const uint64_t q = (k0_ - index) * steps_h_[ch];  // mod 2^64: the phase difference as Q0.64
      const long double a = static_cast<long double>(q) / 18446744073709551616.0L * 6.283185307179586476925L;
      const long double c = std::cos(a), sn = std::sin(a);
      for (int t = 0; t < kWbfmHist; ++t) {
        f2& v = h[static_cast<size_t>(ch) * kWbfmHist + t];
        const long double re = v.x, im = v.y;
        v.x = static_cast<float>(re * c - im * sn);
        v.y = static_cast<float>(re * sn + im * c);
      }
    }
    ORION_HIP(hipMemcpy(hist_[cur_].as<void>(), h.data(), h.size() * sizeof(f2), hipMemcpyHostToDevice));
  }
  int set_path(int path, int max_seg) {
    if ((path != kPathAuto && path != kPathSeg && path != kPathSplit && path != kPathGraph) || max_seg < 0) return -3;
    if (path == kPathSeg && !seg_ok_) return -3;
    if (path == kPathSplit && !split_ok_) return -3;
    if (path != path_) {
      if (processed_) return -3;  // the paths carry their state differently: choose before the first call
      stages_.clear();
    }
    path_ = path;
    max_seg_ = max_seg;
    return 0;
  }

 private:
  int resolved_path() const {
    if (path_ != kPathAuto) return path_;
    return seg_ok_ ? kPathSeg : split_ok_ ? kPathSplit : kPathGraph;
  }
  // ---- fused paths: constants ----
  void build_fused(const std::vector<float>& f_off) {
    const WbfmParams& p = p_;
    const float fs2 = p.fs / static_cast<float>(p.m);
    std::memset(&cf_, 0, sizeof(cf_));
    std::memset(&cb_, 0, sizeof(cb_));
    const auto g = fir_lowpass_as_standard(h_dec_);
    for (size_t k = 0; k < g.size(); ++k) cf_.g[(k % 8) * kWbfmQ + k / 8] = g[k];
    cf_.k = 1.0f / std::max(p.dev_hz, 1.0f);  // fm.rs:23
    const auto a = fir_lowpass_as_standard(h_aud_);
    for (size_t k = 0; k < a.size(); ++k) cb_.a[k] = a[k];
    const BiquadCoeffs bq = lp_cascade_design(fs2, p.audio_bw * 0.9f);  // fm.rs:24
    cb_.b0 = bq.b0; cb_.b1 = bq.b1; cb_.b2 = bq.b2; cb_.a1 = bq.a1; cb_.a2 = bq.a2;
    const StateSpace ss = lp_cascade_ss(bq);
    auto pwm = mat_pow(ss.A, 4, kBackC);
    for (int s = 0; s < 6; ++s) {
      for (int i = 0; i < 16; ++i) cb_.pw[s * 16 + i] = pwm[i];
      pwm = mat_mul(pwm, pwm, 4);
    }
    const auto mw = mat_pow(ss.A, 4, 64ull * kBackC);
    for (int i = 0; i < 16; ++i) cb_.mw[i] = mw[i];
    std::vector<double> lm(64 * 16);
    for (int L = 0; L < 64; ++L) {
      const auto m = mat_pow(ss.A, 4, static_cast<uint64_t>(kBackC) * L);
      std::copy(m.begin(), m.end(), lm.begin() + L * 16);
    }
    lanemats_.upload(lm.data(), lm.size() * sizeof(double));
    // segmented chain constants: steps A^(kSgC 2^s), and A^(kSgL/2)
    std::memset(&cs_, 0, sizeof(cs_));
    cs_.b0 = bq.b0; cs_.b1 = bq.b1; cs_.b2 = bq.b2; cs_.a1 = bq.a1; cs_.a2 = bq.a2;
    std::vector<double> mats(kWbfmMats);
    auto ps = mat_pow(ss.A, 4, kSgC);
    for (int s = 0; s < 6; ++s) {
      for (int i = 0; i < 16; ++i) mats[s * 16 + i] = ps[i];
      ps = mat_mul(ps, ps, 4);
    }
    const auto msh = mat_pow(ss.A, 4, kSgL / 2);
    for (int i = 0; i < 16; ++i) mats[6 * 16 + i] = msh[i];
    mats_.upload(mats.data(), mats.size() * sizeof(double));
    cs_.mats = mats_.as<double>();
    build_audio_frags(a);
    // The segmented chain starts every segment's first sub-range from a zero state and
    // hands the next sub-range that sub-range's zero-state end state and last 128
    // outputs: exact when A^(kSgL - 128) is below f32 resolution relative to A^0 = I
    // (~1e-16 for the WBFM defaults). The split path's back starts each half from a
    // kBackW-sample zero-state warm-up: the same test on A^kBackW.
    auto fro = [&](uint64_t k) {
      const auto m = mat_pow(ss.A, 4, k);
      double f = 0.0;
      for (double v : m) f += v * v;
      return std::sqrt(f);
    };
    seg_ok_ = fro(kSgL - 128) < 1e-10;
    split_ok_ = fro(kBackW) < 1e-7;  // the WBFM defaults: 2.0e-8
    std::vector<uint64_t> steps(nch_);
    std::vector<float> tabs;
    tabs.reserve(static_cast<size_t>(nch_) * kWbfmNS * 2);
    for (int ch = 0; ch < nch_; ++ch) {
      const Oscillator o = oscillator(-f_off[ch], p.fs);  // Rotator::new(-f_off, fs)
      const double th = rec_mean_step(o.w_re, o.w_im, o.step_q64);
      steps[ch] = q64_of_angle(th);
      const auto t = phasor_table(th, kWbfmNS);
      tabs.insert(tabs.end(), t.begin(), t.end());
    }
    step_.upload(steps.data(), steps.size() * sizeof(uint64_t));
    steps_h_ = steps;
    tab_.upload(tabs.data(), tabs.size() * sizeof(float));
  }
  // The segmented chain's audio FIR runs on f16 matrix cores with hi + lo parts
  // (k_wbfm.hip sg::back): the A fragments of the Toeplitz tap matrix, the taps scaled
  // by 2^st so that max |a| 2^st lies in [2^14, 2^15) (a power of two: exact). The f
  // scale is the kernel's, per sub-range.
  void build_audio_frags(const std::vector<float>& a) {
#if ORION_WBFM_EXACT_FIR
    cs_.tscale = 1.0f;
    std::vector<float> at(kAudFragBytes / 4, 0.0f);
    for (int m = 0; m < 176; ++m) {
      const int k = m - 31;
      if (k >= 0 && k < 128 && k < static_cast<int>(a.size())) at[m] = a[k];
    }
    afrag_.upload(at.data(), kAudFragBytes);
    return;
#endif
    float amax = 0.0f;
    for (float v : a) amax = std::max(amax, std::fabs(v));
    int e = 0;
    (void)std::frexp(amax, &e);  // amax < 2^e
    const int st2 = amax > 0.0f ? std::max(-100, std::min(100, 15 - e)) : 0;
    cs_.tscale = std::ldexp(1.0f, -st2);
    // r[u] = a[127 - u] 2^st for u in [0, 128), 0 elsewhere; A[I][kap] = a[I + 128 - kap]
    // = r[kap - I - 1] (kernels.hpp kAudTapWords)
    auto r = [&](int u, int part) -> _Float16 {
      const int k = 127 - u;
      const float v = (u >= 0 && u < 128 && k < static_cast<int>(a.size())) ? std::ldexp(a[k], st2) : 0.0f;
      const _Float16 h = static_cast<_Float16>(v);
      return part == 0 ? h : static_cast<_Float16>(v - static_cast<float>(h));
    };
    std::vector<_Float16> fr(kAudFragBytes / 2);
    for (int part = 0; part < 2; ++part)
      for (int p = 0; p < 2; ++p)
        for (int w = 0; w < kAudTapWords; ++w) {
          _Float16* d = fr.data() + ((part * 2 + p) * kAudTapWords + w) * 2;
          d[0] = r(2 * w - 16 - p, part);
          d[1] = r(2 * w - 15 - p, part);
        }
    afrag_.upload(fr.data(), kAudFragBytes);
  }
  // ---- graph path: the reference's four blocks, per channel ----
  struct Stages {
    std::unique_ptr<Block> rot, dec, fm, aud;
  };
  void graph(const f2* x, size_t n, float* y, size_t out_cap, size_t n_dec, hipStream_t s) {
    const WbfmParams& p = p_;
    const float fs2 = p.fs / static_cast<float>(p.m);
    if (stages_.empty()) {
      for (int ch = 0; ch < nch_; ++ch) {
        Stages st;
        st.rot = make_rotator(-f_off_[ch], p.fs);
        if (seek_) osc_seek(st.rot.get(), seek_);
        st.dec = make_fir_decimator(p.fs, p.m, p.dec_cutoff, p.dec_trans, 1);
        st.fm = make_fm_demod(fs2, p.dev_hz, p.audio_bw);
        st.aud = make_fir_lowpass(fs2, p.audio_pass, p.audio_trans);
        stages_.push_back(std::move(st));
      }
    }
    const size_t nd_all = out_len(n);
    mixed_.resize(n * sizeof(f2));
    dec_.resize(std::max<size_t>(1, nd_all) * sizeof(f2));
    phi_.resize(std::max<size_t>(1, nd_all) * sizeof(float));
    for (int ch = 0; ch < nch_; ++ch) {
      Stages& st = stages_[ch];
      const f2* xc = x + static_cast<size_t>(ch) * n;
      st.rot->process_device(xc, n, mixed_.as<void>(), n, s);
      // decim.rs:44-76: all input consumed, min(ceil(n/m), cap) written
      const WorkReport wd = st.dec->process_device(mixed_.as<void>(), n, dec_.as<void>(), n_dec, s);
      st.fm->process_device(dec_.as<void>(), wd.out_written, phi_.as<void>(), wd.out_written, s);
      st.aud->process_device(phi_.as<void>(), wd.out_written, y + static_cast<size_t>(ch) * out_cap, out_cap, s);
    }
  }

  WbfmParams p_;
  int nch_;
  std::vector<float> f_off_;
  std::vector<float> h_dec_, h_aud_;
  WbfmFrontConst cf_{};
  WbfmBackConst cb_{};
  WbfmFusedConst cs_{};
  bool fused_ok_ = false, seg_ok_ = false, split_ok_ = false;
  int path_ = kPathAuto, max_seg_ = 0;
  uint32_t epoch_ = 0;
  DevBuf step_, tab_, carry_[2], hist_[2], lanemats_, phi_, hand_, flags_, trace_, afrag_, mixed_, dec_, mats_;
  std::vector<Stages> stages_;
  uint64_t seek_ = 0;
  std::vector<uint64_t> steps_h_;  // the fused paths' per-channel mixer steps (Q0.64)
  int cur_ = 0;
  uint64_t k0_ = 0;
  bool processed_ = false;  // a call has run since construction or reset()
};

}  // namespace

std::unique_ptr<Block> make_rotator(float f, float fs) { return std::make_unique<RotatorBlock>(f, fs); }
std::unique_ptr<Block> make_nco(float f, float fs) { return std::make_unique<NcoBlock>(f, fs); }
int osc_set_freq(Block* b, const char* kind, float f, float fs) {
  auto* o = dynamic_cast<OscBlock*>(b);
  if (!o || std::strcmp(b->name(), kind) != 0) return -4;
  // Nco::set_freq keeps the fs it was built with (nco.rs:33-38); Rotator::set_freq takes
  // one (rotator.rs:35-39): a non-finite step (fs = 0) is rejected (ORION_E_ARG).
  o->set_freq(f, std::strcmp(kind, "Nco") == 0 ? o->fs() : fs);
  return 0;
}
int osc_reset_phase(Block* b) {
  auto* o = dynamic_cast<RotatorBlock*>(b);
  if (!o) return -4;
  o->reset();
  return 0;
}
int osc_mix_usb(Block* b, const void* in, size_t n, float* out, hipStream_t s) {
  auto* o = dynamic_cast<RotatorBlock*>(b);
  if (!o) return -4;
  o->run(1, in, out, n, s);
  return 0;
}
int osc_seek(Block* b, uint64_t index) {
  auto* o = dynamic_cast<OscBlock*>(b);
  if (!o) return -4;
  o->seek(index);
  return 0;
}
int osc_next_cs(Block* b, const char* kind, void* out, size_t n, hipStream_t s) {
  auto* o = dynamic_cast<OscBlock*>(b);
  if (!o || std::strcmp(b->name(), kind) != 0) return -4;
  o->run(3, nullptr, out, n, s);
  return 0;
}
std::unique_ptr<Block> make_am_mod(float fs, float rf_hz, float cl, float mi) {
  return std::make_unique<AmModBlock>(fs, rf_hz, cl, mi);
}
std::unique_ptr<Block> make_fm_mod(float fs, float dev_hz, float rf_hz) {
  return std::make_unique<FmModBlock>(fs, dev_hz, rf_hz);
}
int mod_set_gain(Block* b, float g) {
  if (auto* a = dynamic_cast<AmModBlock*>(b)) { a->set_gain(g); return 0; }
  if (auto* f = dynamic_cast<FmModBlock*>(b)) { f->set_gain(g); return 0; }
  if (auto* p = dynamic_cast<PmModBlock*>(b)) { p->set_gain(g); return 0; }
  return cw_mod_set_gain(b, g);
}
std::unique_ptr<Block> make_pm_mod(float fs, float kp, float rf_hz) { return std::make_unique<PmModBlock>(fs, kp, rf_hz); }
int pm_mod_set_sensitivity(Block* b, float kp) {
  auto* p = dynamic_cast<PmModBlock*>(b);
  if (!p) return -4;
  p->set_sensitivity(kp);
  return 0;
}
int am_mod_set_clamp(Block* b, bool on) {
  auto* a = dynamic_cast<AmModBlock*>(b);
  if (!a) return -4;
  a->set_clamp(on);
  return 0;
}
int fm_mod_set_deviation(Block* b, float d) {
  auto* f = dynamic_cast<FmModBlock*>(b);
  if (!f) return -4;
  f->set_deviation(d);
  return 0;
}
std::unique_ptr<Block> make_fir_decimator(float fs, size_t m, float cutoff, float trans, int nch) {
  return std::make_unique<DecimBlock>(fs, m, cutoff, trans, nch);
}
std::unique_ptr<Block> make_fir_lowpass(float fs, float pass, float trans) {
  return std::make_unique<FirRealBlock>(fs, pass, trans);
}
std::unique_ptr<Block> make_fir_lowpass_iq(const std::vector<float>& taps, int nch) {
  return std::make_unique<FirIqBlock>(taps, nch);
}
int fir_lowpass_iq_filter_aligned(Block* b, void* io, size_t n, hipStream_t s) {
  auto* f = dynamic_cast<FirIqBlock*>(b);
  if (!f) return -4;
  f->aligned(io, n, s);
  return 0;
}
std::unique_ptr<Block> make_wbfm_chain(const WbfmParams& p, const std::vector<float>& f_off) {
  return std::make_unique<WbfmBlock>(p, f_off);
}
int wbfm_chain_configure(Block* b, int path, int max_segments) {
  auto* w = dynamic_cast<WbfmBlock*>(b);
  if (!w) return -4;
  return w->set_path(path, max_segments);
}

int wbfm_chain_seek(Block* b, unsigned long long index) {
  auto* w = dynamic_cast<WbfmBlock*>(b);
  if (!w) return -4;
  w->seek(index);
  return 0;
}

}  // namespace orion
