// capi.cpp — extern "C" boundary (include/orion_sdr_amd.h) over the Block layer.
#include "../../include/orion_sdr_amd.h"

#include <algorithm>
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <vector>

#include "blocks.hpp"
#include "osc.hpp"
#include "scan_blocks.hpp"

struct orion_block {
  std::unique_ptr<orion::Block> impl;
};

namespace {
thread_local std::string g_err;

int fail(int code, const char* what) {
  g_err = what ? what : "unknown error";
  return code;
}

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const orion::HipError& e) {
    return fail(ORION_E_HIP, e.what());
  } catch (const std::invalid_argument& e) {
    return fail(ORION_E_ARG, e.what());
  } catch (const std::exception& e) {
    return fail(ORION_E_HIP, e.what());
  }
}

template <class F>
orion_block* make(F&& f) {
  try {
    auto b = new orion_block;
    b->impl = f();
    return b;
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}
}  // namespace

extern "C" {

const char* orion_version(void) { return "orion-sdr-amd 0.1.0 (gfx950)"; }
const char* orion_last_error(void) { return g_err.c_str(); }

int orion_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
int orion_set_device(int d) {
  return guarded([&] {
    ORION_HIP(hipSetDevice(d));
    return ORION_OK;
  });
}
size_t orion_diag_stream_read_bytes(size_t bytes) {
  try {
    return static_cast<size_t>(orion::stream_read_bytes(static_cast<long long>(bytes)));
  } catch (...) {
    return 0;
  }
}
int orion_diag_stream_read(const void* dev, size_t bytes, void* stream) {
  if (!dev) return fail(ORION_E_NULL, "null buffer");
  if (reinterpret_cast<uintptr_t>(dev) % 16) return fail(ORION_E_ARG, "buffer not 16-B aligned");
  return guarded([&] {
    static orion::DevBuf sink(256);
    orion::launch_stream_read(dev, static_cast<long long>(bytes), sink.as<float>(),
                              static_cast<hipStream_t>(stream));
    return ORION_OK;
  });
}
void* orion_host_alloc(size_t bytes) {
  try {
    return orion::host_alloc(bytes);
  } catch (const std::exception& e) {
    fail(ORION_E_HIP, e.what());
    return nullptr;
  }
}
int orion_host_free(void* p) {
  return guarded([&] {
    orion::host_free(p);
    return ORION_OK;
  });
}
int orion_device_cus(void) {
  try {
    return orion::device_cus();
  } catch (const std::exception& e) {
    return fail(ORION_E_HIP, e.what());
  }
}
int orion_diag_spin(void* stream, uint32_t workgroups, uint32_t lds_bytes, double seconds) {
  return guarded([&] {
    orion::launch_spin(static_cast<int>(workgroups), static_cast<int>(lds_bytes), seconds,
                       static_cast<hipStream_t>(stream));
    return ORION_OK;
  });
}
void* orion_diag_stream_create(uint32_t n_cus) {
  hipStream_t st = nullptr;
  try {
    if (n_cus == 0) {
      ORION_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    } else {
      const int ncu = orion::device_cus();
      std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
      for (uint32_t c = 0; c < n_cus && c < static_cast<uint32_t>(ncu); ++c) mask[c / 32] |= 1u << (c % 32);
      ORION_HIP(hipExtStreamCreateWithCUMask(&st, static_cast<uint32_t>(mask.size()), mask.data()));
    }
  } catch (const std::exception& e) {
    fail(ORION_E_HIP, e.what());
    return nullptr;
  }
  return st;
}
int orion_diag_stream_destroy(void* stream) {
  if (!stream) return fail(ORION_E_NULL, "null stream");
  return guarded([&] {
    ORION_HIP(hipStreamDestroy(static_cast<hipStream_t>(stream)));
    return ORION_OK;
  });
}
int orion_synchronize(void* stream) {
  return guarded([&] {
    ORION_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return ORION_OK;
  });
}

orion_block* orion_rotator_new(float freq_hz, float fs) {
  return make([&] { return orion::make_rotator(freq_hz, fs); });
}
orion_block* orion_nco_new(float freq_hz, float fs) {
  return make([&] { return orion::make_nco(freq_hz, fs); });
}
int orion_rotator_set_freq(orion_block* b, float freq_hz, float fs) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    if (orion::osc_set_freq(b->impl.get(), "Rotator", freq_hz, fs)) return fail(ORION_E_TYPE, "not a Rotator");
    return ORION_OK;
  });
}
int orion_rotator_reset_phase(orion_block* b) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    if (orion::osc_reset_phase(b->impl.get())) return fail(ORION_E_TYPE, "not a Rotator");
    return ORION_OK;
  });
}
int orion_rotator_mix_usb_block_device(orion_block* b, const void* in, size_t n_in, float* out, size_t out_cap,
                                       void* stream, orion_work_report* wr) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  if ((!in && n_in) || (!out && out_cap)) return fail(ORION_E_NULL, "null buffer");
  return guarded([&] {
    b->impl->check_device_errors();
    const size_t n = std::min(n_in, out_cap);  // rotator.rs:89
    if (orion::osc_mix_usb(b->impl.get(), in, n, out, static_cast<hipStream_t>(stream)))
      return fail(ORION_E_TYPE, "not a Rotator");
    if (wr) { wr->in_read = n; wr->out_written = n; }
    return ORION_OK;
  });
}
int orion_rotator_mix_usb_block(orion_block* b, const void* in, size_t n_in, float* out, size_t out_cap,
                                orion_work_report* wr) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  if ((!in && n_in) || (!out && out_cap)) return fail(ORION_E_NULL, "null buffer");
  return guarded([&] {
    const size_t n = std::min(n_in, out_cap);
    orion::DevBuf di(n * 8 + 16), dout(n * 4 + 16);
    if (n) ORION_HIP(hipMemcpy(di.as<void>(), in, n * 8, hipMemcpyHostToDevice));
    if (orion::osc_mix_usb(b->impl.get(), di.as<void>(), n, dout.as<float>(), nullptr))
      return fail(ORION_E_TYPE, "not a Rotator");
    if (n) ORION_HIP(hipMemcpy(out, dout.as<void>(), n * 4, hipMemcpyDeviceToHost));
    ORION_HIP(hipDeviceSynchronize());
    if (wr) { wr->in_read = n; wr->out_written = n; }
    return ORION_OK;
  });
}
int orion_nco_set_freq(orion_block* b, float freq_hz) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    if (orion::osc_set_freq(b->impl.get(), "Nco", freq_hz, 0.0f)) return fail(ORION_E_TYPE, "not an Nco");
    return ORION_OK;
  });
}
namespace {
int next_cs_device(orion_block* b, const char* kind, void* out, size_t n, void* stream) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  if (!out && n) return fail(ORION_E_NULL, "null buffer");
  return guarded([&] {
    b->impl->check_device_errors();
    if (orion::osc_next_cs(b->impl.get(), kind, out, n, static_cast<hipStream_t>(stream)))
      return fail(ORION_E_TYPE, "wrong oscillator kind");
    return ORION_OK;
  });
}
int next_cs_host(orion_block* b, const char* kind, void* out, size_t n) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  if (!out && n) return fail(ORION_E_NULL, "null buffer");
  return guarded([&] {
    orion::DevBuf d(n * 8 + 16);
    if (orion::osc_next_cs(b->impl.get(), kind, d.as<void>(), n, nullptr)) return fail(ORION_E_TYPE, "wrong oscillator kind");
    if (n) ORION_HIP(hipMemcpy(out, d.as<void>(), n * 8, hipMemcpyDeviceToHost));
    ORION_HIP(hipDeviceSynchronize());
    return ORION_OK;
  });
}
}  // namespace
int orion_nco_next_cs_block_device(orion_block* b, void* out, size_t n, void* stream) {
  return next_cs_device(b, "Nco", out, n, stream);
}
int orion_nco_next_cs_block(orion_block* b, void* out, size_t n) { return next_cs_host(b, "Nco", out, n); }
int orion_rotator_next_cs_block_device(orion_block* b, void* out, size_t n, void* stream) {
  return next_cs_device(b, "Rotator", out, n, stream);
}
int orion_rotator_next_cs_block(orion_block* b, void* out, size_t n) { return next_cs_host(b, "Rotator", out, n); }
orion_block* orion_fir_decimator_new(float fs, size_t m, float cutoff_hz, float trans_hz) {
  return make([&] { return orion::make_fir_decimator(fs, m, cutoff_hz, trans_hz, 1); });
}
orion_block* orion_fir_decimator_batch_new(float fs, size_t m, float cutoff_hz, float trans_hz, size_t nch) {
  return make([&] { return orion::make_fir_decimator(fs, m, cutoff_hz, trans_hz, static_cast<int>(nch)); });
}
orion_block* orion_fir_lowpass_new(float fs, float pass_hz, float trans_hz) {
  return make([&] { return orion::make_fir_lowpass(fs, pass_hz, trans_hz); });
}
orion_block* orion_fir_lowpass_iq_design(size_t num_taps, float cutoff_norm, float stopband_db) {
  return make([&] { return orion::make_fir_lowpass_iq(orion::kaiser_lowpass_taps(num_taps, cutoff_norm, stopband_db)); });
}
orion_block* orion_fir_lowpass_iq_from_taps(const float* taps, size_t n) {
  return make([&] { return orion::make_fir_lowpass_iq(std::vector<float>(taps, taps + (taps ? n : 0))); });
}
orion_block* orion_fir_lowpass_iq_batch_from_taps(const float* taps, size_t n, size_t nch) {
  return make([&] {
    if (nch < 1 || nch > (1u << 16)) throw std::invalid_argument("FirLowpassIq batch: 1 <= nch <= 65536");
    return orion::make_fir_lowpass_iq(std::vector<float>(taps, taps + (taps ? n : 0)), static_cast<int>(nch));
  });
}
int orion_osc_table_phasors(float freq_hz, float fs, uint64_t max_out, void* out, size_t n, uint64_t* cyc_start,
                            uint64_t* cyc_len, uint64_t* n_tab) {
  if (!out && n) return fail(ORION_E_NULL, "null buffer");
  return guarded([&] {
    if (max_out > orion::kNcoTableMax) return fail(ORION_E_ARG, "budget above 2^28");
    const orion::Oscillator o = orion::oscillator(freq_hz, fs);
    const orion::RecTable t = orion::rec_table(o.w_re, o.w_im, orion::RecState{}, max_out, orion::kOscSpan, o.step_q64);
    float* z = static_cast<float*>(out);
    for (size_t k = 0; k < n; ++k) {
      const orion::RecState st = orion::rec_state_after(t, k);
      z[2 * k] = st.zr;
      z[2 * k + 1] = st.zi;
    }
    if (cyc_start) *cyc_start = t.cyc_start;
    if (cyc_len) *cyc_len = t.cyc_len;
    if (n_tab) *n_tab = t.n;
    return ORION_OK;
  });
}
int orion_fir_lowpass_iq_num_taps(const orion_block* b, size_t* n) {
  if (!b || !n) return fail(ORION_E_NULL, "null argument");
  if (std::strcmp(b->impl->name(), "FirLowpassIq") != 0) return fail(ORION_E_TYPE, "not a FirLowpassIq");
  *n = b->impl->taps(0).size();  // fir.rs:210-212 taps.len()
  return ORION_OK;
}
int orion_fir_lowpass_iq_group_delay(const orion_block* b, size_t* d) {
  size_t n = 0;
  const int rc = orion_fir_lowpass_iq_num_taps(b, &n);
  if (rc) return rc;
  *d = (n - 1) / 2;  // fir.rs:216-218 (taps.len() - 1) / 2; from_taps keeps len >= 1
  return ORION_OK;
}
int orion_fir_lowpass_iq_filter_aligned_device(orion_block* b, void* io, size_t n, void* stream) {
  if (!b || (!io && n)) return fail(ORION_E_NULL, "null argument");
  return guarded([&] { return orion::fir_lowpass_iq_filter_aligned(b->impl.get(), io, n, static_cast<hipStream_t>(stream)); });
}
int orion_fir_lowpass_iq_filter_aligned(orion_block* b, void* io, size_t n) {
  if (!b || (!io && n)) return fail(ORION_E_NULL, "null argument");
  return guarded([&] {
    orion::DevBuf d(n * 8 + 8);
    if (n) ORION_HIP(hipMemcpy(d.as<void>(), io, n * 8, hipMemcpyHostToDevice));
    const int rc = orion::fir_lowpass_iq_filter_aligned(b->impl.get(), d.as<void>(), n, nullptr);
    if (rc) return rc;
    if (n) ORION_HIP(hipMemcpy(io, d.as<void>(), n * 8, hipMemcpyDeviceToHost));
    ORION_HIP(hipDeviceSynchronize());
    return ORION_OK;
  });
}
orion_block* orion_agc_rms_new(float fs, float attack_ms, float release_ms, float target_rms) {
  return make([&] { return orion::make_agc(false, fs, attack_ms, release_ms, target_rms); });
}
orion_block* orion_agc_rms_iq_new(float fs, float attack_ms, float release_ms, float target_rms) {
  return make([&] { return orion::make_agc(true, fs, attack_ms, release_ms, target_rms); });
}
orion_block* orion_am_dsb_mod_new(float fs, float rf_hz, float carrier_level, float modulation_index) {
  return make([&] { return orion::make_am_mod(fs, rf_hz, carrier_level, modulation_index); });
}
int orion_am_dsb_mod_set_gain(orion_block* b, float g) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  if (std::strcmp(b->impl->name(), "AmDsbMod") != 0) return fail(ORION_E_TYPE, "not an AmDsbMod");
  return guarded([&] { return orion::mod_set_gain(b->impl.get(), g); });
}
int orion_am_dsb_mod_set_clamp(orion_block* b, int on) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    if (orion::am_mod_set_clamp(b->impl.get(), on != 0)) return fail(ORION_E_TYPE, "not an AmDsbMod");
    return ORION_OK;
  });
}
orion_block* orion_fm_phase_accum_mod_new(float fs, float deviation_hz, float rf_hz) {
  return make([&] { return orion::make_fm_mod(fs, deviation_hz, rf_hz); });
}
int orion_fm_phase_accum_mod_set_deviation(orion_block* b, float deviation_hz) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    if (orion::fm_mod_set_deviation(b->impl.get(), deviation_hz)) return fail(ORION_E_TYPE, "not an FmPhaseAccumMod");
    return ORION_OK;
  });
}
int orion_fm_phase_accum_mod_set_gain(orion_block* b, float g) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  if (std::strcmp(b->impl->name(), "FmPhaseAccumMod") != 0) return fail(ORION_E_TYPE, "not an FmPhaseAccumMod");
  return guarded([&] { return orion::mod_set_gain(b->impl.get(), g); });
}
orion_block* orion_pm_direct_phase_mod_new(float fs, float kp_rad_per_unit, float rf_hz) {
  return make([&] { return orion::make_pm_mod(fs, kp_rad_per_unit, rf_hz); });
}
int orion_pm_direct_phase_mod_set_gain(orion_block* b, float g) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  if (std::strcmp(b->impl->name(), "PmDirectPhaseMod") != 0) return fail(ORION_E_TYPE, "not a PmDirectPhaseMod");
  return guarded([&] { return orion::mod_set_gain(b->impl.get(), g); });
}
int orion_pm_direct_phase_mod_set_sensitivity(orion_block* b, float kp_rad_per_unit) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    if (orion::pm_mod_set_sensitivity(b->impl.get(), kp_rad_per_unit)) return fail(ORION_E_TYPE, "not a PmDirectPhaseMod");
    return ORION_OK;
  });
}
orion_block* orion_cw_keyed_mod_new(float fs, float tone_hz, float rise_ms, float fall_ms) {
  return make([&] { return orion::make_cw_mod(fs, tone_hz, rise_ms, fall_ms); });
}
int orion_cw_keyed_mod_set_gain(orion_block* b, float g) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    if (orion::cw_mod_set_gain(b->impl.get(), g)) return fail(ORION_E_TYPE, "not a CwKeyedMod");
    return ORION_OK;
  });
}
orion_block* orion_ssb_phasing_mod_new(float fs, float audio_bw_hz, float audio_if_hz, float rf_hz, int usb) {
  return make([&] { return orion::make_ssb_mod(fs, audio_bw_hz, audio_if_hz, rf_hz, usb != 0); });
}
orion_block* orion_lp_cascade_new(float fs, float fc) {
  return make([&] { return orion::make_lp_cascade(fs, fc); });
}
orion_block* orion_biquad_new(float b0, float b1, float b2, float a1, float a2) {
  return make([&] { return orion::make_biquad(b0, b1, b2, a1, a2); });
}
orion_block* orion_lp_dc_cascade_new(float fs, float lp_fc, float dc_cut_hz) {
  return make([&] { return orion::make_lp_dc_cascade(fs, lp_fc, dc_cut_hz); });
}
int orion_lp_dc_cascade_set_map(orion_block* b, int map) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    const int rc = orion::lp_dc_cascade_set_map(b->impl.get(), map);
    if (rc == -4) return fail(ORION_E_TYPE, "not an LpDcCascade");
    if (rc == -3) return fail(ORION_E_ARG, "unknown process_mapped map (ORION_MAP_IDENTITY / SQRT / ABS)");
    return ORION_OK;
  });
}
int orion_lp_dc_cascade_set_sqrt_map(orion_block* b, int on) {
  return orion_lp_dc_cascade_set_map(b, on ? ORION_MAP_SQRT : ORION_MAP_IDENTITY);
}
orion_block* orion_dc_blocker_new(float fs, float cut_hz) {
  return make([&] { return orion::make_dc_blocker(fs, cut_hz); });
}
orion_block* orion_fm_quadrature_demod_new(float fs, float dev_hz, float audio_bw_hz) {
  return make([&] { return orion::make_fm_demod(fs, dev_hz, audio_bw_hz); });
}
int orion_fm_quadrature_demod_with_translate(orion_block* b, float freq_hz) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] { return orion::fm_demod_with_translate(b->impl.get(), freq_hz); });
}
orion_block* orion_pm_quadrature_demod_new(float fs, float k, float audio_bw_hz) {
  return make([&] { return orion::make_pm_demod(fs, k, audio_bw_hz); });
}
orion_block* orion_ssb_product_demod_new(float fs, float bfo_hz, float audio_bw_hz) {
  return make([&] { return orion::make_ssb_demod(fs, bfo_hz, audio_bw_hz, 1); });
}
orion_block* orion_ssb_product_demod_batch_new(float fs, float bfo_hz, float audio_bw_hz, size_t nch) {
  return make([&] { return orion::make_ssb_demod(fs, bfo_hz, audio_bw_hz, static_cast<int>(nch)); });
}
orion_block* orion_am_envelope_demod_new(float fs, float audio_bw_hz) {
  return make([&] { return orion::make_am_demod(fs, audio_bw_hz); });
}
int orion_am_envelope_demod_with_abs_approx(orion_block* b, float k1, float k2) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] { return orion::am_demod_with_abs_approx(b->impl.get(), k1, k2); });
}
orion_block* orion_cw_envelope_demod_new(float fs, float tone_hz, float env_bw_hz) {
  return make([&] { return orion::make_cw_demod(fs, tone_hz, env_bw_hz); });
}
int orion_cw_envelope_demod_set_gain(orion_block* b, float g) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] { return orion::cw_demod_set_gain(b->impl.get(), g); });
}

static orion::WbfmParams wbfm_params(const orion_wbfm_params* p) {
  return {p->fs, p->dec_cutoff, p->dec_trans, p->dev_hz, p->audio_bw, p->audio_pass, p->audio_trans, p->m};
}
orion_block* orion_wbfm_chain_new(const orion_wbfm_params* p) {
  if (!p) { g_err = "null params"; return nullptr; }
  return make([&] { return orion::make_wbfm_chain(wbfm_params(p), {p->f_off}); });
}
orion_block* orion_wbfm_chain_batch_new(const orion_wbfm_params* p, const float* f_off, size_t nch) {
  if (!p || !f_off || nch == 0) { g_err = "null params / no channels"; return nullptr; }
  return make([&] { return orion::make_wbfm_chain(wbfm_params(p), std::vector<float>(f_off, f_off + nch)); });
}

int orion_wbfm_chain_configure(orion_block* b, int path, int max_segments) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    const int rc = orion::wbfm_chain_configure(b->impl.get(), path, max_segments);
    if (rc == -4) return fail(ORION_E_TYPE, "not a WBFM chain");
    if (rc != 0) return fail(ORION_E_ARG, "WBFM path unavailable for this design (or bad arguments)");
    return ORION_OK;
  });
}

int orion_wbfm_chain_seek(orion_block* b, uint64_t index) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    if (orion::wbfm_chain_seek(b->impl.get(), index) == -4) return fail(ORION_E_TYPE, "not a WBFM chain");
    return ORION_OK;
  });
}

int orion_block_process(orion_block* b, const void* in, size_t n_in, void* out, size_t out_cap,
                        orion_work_report* wr) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  if ((!in && n_in) || (!out && out_cap)) return fail(ORION_E_NULL, "null buffer");
  return guarded([&] {
    const orion::WorkReport w = b->impl->process_host(in, n_in, out, out_cap);
    if (wr) { wr->in_read = w.in_read; wr->out_written = w.out_written; }
    return ORION_OK;
  });
}
int orion_block_process_device(orion_block* b, const void* in, size_t n_in, void* out, size_t out_cap,
                               void* stream, orion_work_report* wr) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  if ((!in && n_in) || (!out && out_cap)) return fail(ORION_E_NULL, "null buffer");
  return guarded([&] {
    const orion::Block& blk = *b->impl;
    const size_t nch = static_cast<size_t>(blk.channels());
    const size_t ib = nch * n_in * orion::dt_size(blk.in_type()), ob = nch * out_cap * orion::dt_size(blk.out_type());
    const char *ip = static_cast<const char*>(in), *op = static_cast<const char*>(out);
    if (ib && ob && ip < op + ob && op < ip + ib && !blk.alias_ok())
      return fail(ORION_E_ARG, "input and output device ranges overlap (not supported by this block)");
    b->impl->check_device_errors();  // a wait that timed out in an earlier call of this handle
    const orion::WorkReport w = b->impl->process_device(in, n_in, out, out_cap, static_cast<hipStream_t>(stream));
    if (wr) { wr->in_read = w.in_read; wr->out_written = w.out_written; }
    return ORION_OK;
  });
}
int orion_batch_process(orion_block* b, const void* in, size_t n_ch, size_t n_per_ch, void* out, size_t out_cap,
                        void* stream, orion_work_report* wr) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  if (n_ch != static_cast<size_t>(b->impl->channels()))
    return fail(ORION_E_ARG, "n_ch differs from the handle's channel count (build it with a *_batch_new constructor)");
  return orion_block_process_device(b, in, n_per_ch, out, out_cap, stream, wr);
}
int orion_block_configure(orion_block* b, int option, long long value) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    const int rc = b->impl->configure(option, value);
    if (rc == -4) return fail(ORION_E_TYPE, "option not supported by this block");
    if (rc != 0) return fail(ORION_E_ARG, "bad option value");
    return ORION_OK;
  });
}
int orion_block_status(orion_block* b) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    b->impl->check_device_errors();
    return ORION_OK;
  });
}
void orion_debug_set_spin_limit(uint32_t polls) { orion::set_spin_limit(polls); }
uint32_t orion_debug_spin_limit(void) { return orion::spin_limit(); }
int orion_block_reset(orion_block* b) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  return guarded([&] {
    b->impl->reset();
    return ORION_OK;
  });
}
void orion_block_free(orion_block* b) { delete b; }
int orion_block_in_type(const orion_block* b) { return b ? static_cast<int>(b->impl->in_type()) : ORION_E_NULL; }
int orion_block_out_type(const orion_block* b) { return b ? static_cast<int>(b->impl->out_type()) : ORION_E_NULL; }
size_t orion_block_out_len(const orion_block* b, size_t n) { return b ? b->impl->out_len(n) : 0; }
size_t orion_block_channels(const orion_block* b) { return b ? static_cast<size_t>(b->impl->channels()) : 0; }
const char* orion_block_name(const orion_block* b) { return b ? b->impl->name() : ""; }
int orion_block_taps(const orion_block* b, int which, float* out, size_t cap, size_t* n) {
  if (!b) return fail(ORION_E_NULL, "null handle");
  const auto t = b->impl->taps(which);
  if (n) *n = t.size();
  if (out) std::memcpy(out, t.data(), std::min(cap, t.size()) * sizeof(float));
  return ORION_OK;
}

size_t orion_fir_lowpass_design(float fs, float pass_hz, float trans_hz, float* taps, size_t cap) {
  const auto t = orion::fir_lowpass_taps(fs, pass_hz, trans_hz);
  if (taps) std::memcpy(taps, t.data(), std::min(cap, t.size()) * sizeof(float));
  return t.size();
}
size_t orion_kaiser_lowpass_taps(size_t num_taps, float cutoff_norm, float stopband_db, float* taps, size_t cap) {
  const auto t = orion::kaiser_lowpass_taps(num_taps, cutoff_norm, stopband_db);
  if (taps) std::memcpy(taps, t.data(), std::min(cap, t.size()) * sizeof(float));
  return t.size();
}
float orion_kaiser_transition_norm(size_t num_taps, float stopband_db) {
  return orion::kaiser_transition_norm(num_taps, stopband_db);
}
size_t orion_kaiser_num_taps(float transition_norm, float stopband_db) {
  return orion::kaiser_num_taps(transition_norm, stopband_db);
}
static orion::TxLowpassSpec tx_spec(const orion_tx_lowpass* t) { return {t->cutoff_norm, t->num_taps, t->stopband_db}; }
orion_tx_lowpass orion_tx_lowpass_for_null_band(size_t n_fft, size_t occupied_half, size_t num_taps, float stopband_db) {
  const auto s = orion::tx_lowpass_for_null_band(n_fft, occupied_half, num_taps, stopband_db);
  return {s.cutoff_norm, s.num_taps, s.stopband_db};
}
size_t orion_tx_lowpass_taps_for_null_band(size_t n_fft, size_t occupied_half, float stopband_db) {
  return orion::tx_lowpass_taps_for_null_band(n_fft, occupied_half, stopband_db);
}
size_t orion_tx_lowpass_group_delay(const orion_tx_lowpass* t) { return t ? orion::tx_lowpass_group_delay(tx_spec(t)) : 0; }
float orion_tx_lowpass_transition_norm(const orion_tx_lowpass* t) {
  return t ? orion::tx_lowpass_transition_norm(tx_spec(t)) : 0.0f;
}
int orion_tx_lowpass_transition_fits(const orion_tx_lowpass* t, size_t n_fft, size_t occupied_half) {
  return t && orion::tx_lowpass_transition_fits(tx_spec(t), n_fft, occupied_half) ? 1 : 0;
}
float orion_tx_lowpass_stopband_edge_norm(const orion_tx_lowpass* t) {
  return t ? orion::tx_lowpass_stopband_edge_norm(tx_spec(t)) : 0.0f;
}
int orion_tx_lowpass_fits_guard(const orion_tx_lowpass* t, size_t cp_len, size_t roll_off, size_t backoff) {
  return t && orion::tx_lowpass_fits_guard(tx_spec(t), cp_len, roll_off, backoff) ? 1 : 0;
}
orion_block* orion_tx_lowpass_filter(const orion_tx_lowpass* t) {
  if (!t) { g_err = "null spec"; return nullptr; }
  return make([&] { return orion::make_fir_lowpass_iq(orion::kaiser_lowpass_taps(t->num_taps, t->cutoff_norm, t->stopband_db)); });
}
void orion_lp_cascade_design(float fs, float fc, float out5[5]) {
  const auto c = orion::lp_cascade_design(fs, fc);
  out5[0] = c.b0; out5[1] = c.b1; out5[2] = c.b2; out5[3] = c.a1; out5[4] = c.a2;
}

}  // extern "C"
