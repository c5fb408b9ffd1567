// blocks.hpp — C++ mirror of the reference Block contract over the gfx950 kernels.
//
// Reference: trait Block { fn process(&mut self, &[In], &mut [Out]) -> WorkReport }
// (src/core.rs:6-22). Each class owns its device-resident streaming state
// (delay-line history, oscillator sample count, IIR carry, discriminator
// history), so k calls on consecutive chunks equal one call on the
// concatenation — the reference's "resume" semantics.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "design.hpp"
#include "kernels.hpp"

namespace orion {

enum class Dt : int { C32 = 0, F32 = 1 };
// orion_block_configure options (include/orion_sdr_amd.h ORION_OPT_*).
enum : int { kOptScanPath = 1, kOptModPasses = 2, kOptNcoTable = 3 };
inline size_t dt_size(Dt d) { return d == Dt::C32 ? 8 : 4; }

struct WorkReport {
  size_t in_read = 0;
  size_t out_written = 0;
};

// RAII device allocation.
class DevBuf {
 public:
  DevBuf() = default;
  explicit DevBuf(size_t bytes) { resize(bytes); }
  ~DevBuf();
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  void resize(size_t bytes);      // discards contents when it grows
  void zero(hipStream_t s = nullptr);
  void upload(const void* h, size_t bytes, hipStream_t s = nullptr);
  template <class T> T* as() const { return static_cast<T*>(p_); }
  size_t size() const { return n_; }

 private:
  void* p_ = nullptr;
  size_t n_ = 0;
};

class Block {
 public:
  virtual ~Block();
  virtual const char* name() const = 0;
  virtual Dt in_type() const = 0;
  virtual Dt out_type() const = 0;
  // Outputs produced for n inputs when out_cap is unbounded.
  virtual size_t out_len(size_t n_in) const { return n_in; }
  // Device buffers, asynchronous on `s` (no allocation, no sync: graph-capturable
  // once staging has been sized). Channels: blocks built for nch > 1 read
  // in[ch*n_in + i] and write out[ch*out_cap + j].
  virtual WorkReport process_device(const void* in, size_t n_in, void* out, size_t out_cap,
                                    hipStream_t s) = 0;
  // Host buffers (the Block contract a host caller drives, core.rs:12-22), synchronous.
  // Host memory that is pinned (orion_host_alloc / hipHostRegister) moves by DMA
  // directly; pageable memory through two pinned staging buffers per direction, the
  // CPU copy of one chunk overlapping the DMA of the other. Blocks whose output is
  // bitwise independent of how a call is cut (chunk_quantum() > 0: the oscillators,
  // FIRs, decimators, elementwise modulators) run as a pipeline of chunks on three
  // streams (H2D, kernel, D2H overlapped); every other block (the IIR scans, the WBFM
  // chain) uploads the call, runs ONE device call and downloads: in both cases the
  // result equals one orion_block_process_device call on the same input bit for bit.
  WorkReport process_host(const void* in, size_t n_in, void* out, size_t out_cap);
  // Sample granularity at which k calls on consecutive chunks give bit-identical
  // results to one call (0: none; a decimator: m, whose phase restarts every call).
  virtual size_t chunk_quantum() const { return 0; }
  // All n_in inputs are consumed whatever out_cap is (FirDecimator, decim.rs:72-75; the
  // WBFM chain); otherwise n = min(n_in, out_cap) (1:1 blocks).
  virtual bool consumes_all() const { return false; }
  // Errors a kernel flagged in the handle's device error word (a cross-workgroup
  // wait that timed out): throws HipError and clears the word if one is set. The
  // word is host-visible (pinned, coherent), so this needs no sync; it sees every
  // kernel of the handle that has finished (orion_block_status). A composite block
  // (the WBFM chain's graph path) also polls the words of the blocks it owns.
  virtual void check_device_errors();
  virtual void reset() = 0;
  virtual int channels() const { return 1; }
  // process_device may be given overlapping in/out ranges (the block stages its
  // input itself); the C ABI rejects overlap for every other block.
  virtual bool alias_ok() const { return false; }
  // Designed coefficients (for tests): which = 0 primary taps, 1 secondary.
  virtual std::vector<float> taps(int which) const { (void)which; return {}; }
  // Engine options (include/orion_sdr_amd.h orion_block_configure): 0 set, -3 bad
  // value, -4 option not known to this block.
  virtual int configure(int option, long long value) { (void)option; (void)value; return -4; }

 protected:
  hipStream_t host_stream();
  // The handle's device error word (host-pinned, coherent; allocated on first use):
  // kernels set it with system-scope stores, the host reads it without a sync.
  int* dev_err();
  DevBuf stage_in_, stage_out_;

 private:
  struct HostPipe;  // pinned staging, copy streams and events of process_host
  HostPipe& pipe();
  void h2d(void* dst, const void* src, size_t bytes, hipStream_t s);
  void d2h(void* dst, const void* src, size_t bytes, hipStream_t s);
  WorkReport host_chunked(const void* in, size_t n_in, void* out, size_t out_cap, size_t q);
  hipStream_t hs_ = nullptr;
  int* err_ = nullptr;
  HostPipe* pipe_ = nullptr;  // owned (deleted in ~Block, where HostPipe is complete)
};

// Pinned host memory for callers (orion_host_alloc): process_host then moves it by DMA
// without staging copies.
void* host_alloc(size_t bytes);
void host_free(void* p);
bool host_is_pinned(const void* p);

// dsp/rotator.rs:8-95 (rotate_block). C32 -> C32.
std::unique_ptr<Block> make_rotator(float freq_hz, float fs);
// dsp/nco.rs:11-66 (mix_with_nco per sample). C32 -> C32.
std::unique_ptr<Block> make_nco(float freq_hz, float fs);
// Oscillator output index of the next sample (a time shard's phase origin); -4 otherwise.
int osc_seek(Block* b, uint64_t index);
// Oscillator controls (-4 if b is not of that kind): set_freq (Rotator: rotator.rs:35-39,
// kind "Rotator"; Nco: nco.rs:33-38, kind "Nco", the block's own fs), reset_phase
// (rotator.rs:28-31), mix_usb_block (rotator.rs:88-94, C32 -> F32 on device buffers) and
// next / next_cs n times (rotator.rs:44-68 kind "Rotator", nco.rs:42-58 kind "Nco"; C32
// phasors on device buffers), asynchronous on s. set_freq throws std::invalid_argument
// for a non-finite step.
int osc_set_freq(Block* b, const char* kind, float freq_hz, float fs);
int osc_reset_phase(Block* b);
int osc_mix_usb(Block* b, const void* in_dev, size_t n, float* out_dev, hipStream_t s);
int osc_next_cs(Block* b, const char* kind, void* out_dev, size_t n, hipStream_t s);
// dsp/decim.rs:10-77. C32 -> C32, out = ceil(n/m) (decimation phase restarts
// every call, decim.rs:66-71 — reproduced).
std::unique_ptr<Block> make_fir_decimator(float fs, size_t m, float cutoff_hz, float trans_hz,
                                          int nch = 1);
// dsp/fir.rs:7-67. F32 -> F32.
std::unique_ptr<Block> make_fir_lowpass(float fs, float pass_hz, float trans_hz);
// dsp/fir.rs:176-297 (from_taps; empty -> [1.0]). C32 -> C32. nch > 1: independent
// channels sharing the taps (batched [nch][n], as the batched FirDecimator).
std::unique_ptr<Block> make_fir_lowpass_iq(const std::vector<float>& taps, int nch = 1);
// FirLowpassIq::filter_aligned (fir.rs:260-276) on device memory, in place allowed
// via a scratch copy. Resets the block's streaming state first, like the reference.
int fir_lowpass_iq_filter_aligned(Block* b, void* io_dev, size_t n, hipStream_t s);

// Analog modulators. F32 audio -> C32 IQ.
std::unique_ptr<Block> make_am_mod(float fs, float rf_hz, float carrier_level, float modulation_index);  // am.rs
std::unique_ptr<Block> make_fm_mod(float fs, float deviation_hz, float rf_hz);                         // fm.rs
std::unique_ptr<Block> make_pm_mod(float fs, float kp, float rf_hz);                                   // pm.rs
std::unique_ptr<Block> make_cw_mod(float fs, float tone_hz, float rise_ms, float fall_ms);             // cw.rs
int mod_set_gain(Block* b, float g);             // Am / Fm / Pm / Cw modulator set_gain; -4 other blocks
int cw_mod_set_gain(Block* b, float g);          // -4 if not a CwKeyedMod
int pm_mod_set_sensitivity(Block* b, float kp);  // -4 if not a PmDirectPhaseMod
int am_mod_set_clamp(Block* b, bool on);         // -4 if not an AmDsbMod
int fm_mod_set_deviation(Block* b, float d);     // -4 if not an FmPhaseAccumMod
std::unique_ptr<Block> make_agc(bool iq, float fs, float attack_ms, float release_ms, float target_rms);  // agc.rs

// The WBFM chain (docs/demodulate.md:128-133): Rotator(-f_off) -> FirDecimator
// (fs, m, dec_cutoff, dec_trans) -> FmQuadratureDemod(fs/m, dev, audio_bw) ->
// FirLowpass(fs/m, audio_pass, audio_trans). C32 -> F32, out = ceil(n/m).
struct WbfmParams {
  float fs, dec_cutoff, dec_trans, dev_hz, audio_bw, audio_pass, audio_trans;
  size_t m;
};
std::unique_ptr<Block> make_wbfm_chain(const WbfmParams& p, const std::vector<float>& f_off);
// Kernel path of a WBFM chain (tests and timing; include/orion_sdr_amd.h
// orion_wbfm_chain_configure). max_segments > 0 caps the segmented kernel's
// waves (default: the resident capacity). Returns -4 if b is not a WBFM chain,
// -3 if this design cannot run on that path.
enum : int { kPathAuto = 0, kPathSeg = 1, kPathSplit = 3, kPathGraph = 4 };
int wbfm_chain_configure(Block* b, int path, int max_segments);
// Absolute index of the next input sample (the NCO phase origin) of a WBFM
// chain: a time-sharded stream starts each shard's handle at its halo start
// (include/orion_sdr_amd.h orion_wbfm_chain_seek). -4 if b is not a WBFM chain.
int wbfm_chain_seek(Block* b, unsigned long long index);

}  // namespace orion
