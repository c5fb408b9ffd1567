"""bench.py — Msamples/s through the WBFM demod chain on 1..8 MI355X.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`, one process
per GPU under torch.distributed.run for N > 1. A step is one pass of the hot
path over one block of synthetic IQ already resident in HBM: per GPU, one
C2-sized channel (2^26 cf32 @ 10 Msps, its own tuning offset; BASELINE.json
configs[1]). Channels are independent: no collective on the data path
("scaling": "weak"); the only collectives are the timing barrier / max.

The roofline object prices the one kernel the chain runs (k_wbfm_seg) with
HIP events on the stream it is launched on (one pair around the K launches, so
inter-launch gaps count against it): algorithmic bytes per launch
(8 B cf32 in + 4 B f32 audio out per 8 inputs = 8.5 B per input sample, SURVEY
§8d) / average kernel time, against the 8.0 TB/s HBM3E peak. The cpu_baseline
is the scalar oracle ("port" of the reference Rust, 1 thread, the reference is
single-threaded) timed on this host on a bounded prefix of the same input; the
multi-channel configs time the oracle on min(channels, 16) host threads, one
channel per thread, on a bounded prefix of that many channels.

At N = 1 the C2 line also carries "host_fed" (SURVEY §8d's H2D-inclusive figure): the
same chain driven from host memory through orion_block_process, pinned and pageable,
beside the box's raw pinned H2D rate. It is never `value`.

Other workloads (--config c1|c3|c4|c5|c5f) are available for DESIGN.md tables; the
driver's default line is c2. C1 (BASELINE configs[0], the reference's CPU block
graph: 127-tap FirLowpassIq over 2^20 cf32) is compute-bound (508 flop per 16 B),
so its roofline is priced against packed FP32 (157.3 TFLOP/s), not HBM. C5F is
BASELINE configs[4] with its channel filter: a batched 127-tap FirLowpassIq in front
of the batched SsbProductDemod (a two-block device graph), priced on the FIR (FP32).

Multi-process rehearsal on one GPU: --dist-backend gloo and
--device-map 0,0 let two ranks share device 0; --check-shards (C2 stream shards)
gathers every rank's audio to rank 0 and compares it with one call over the stream.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (device memory, streams, torch.distributed: plumbing)

import orion_sdr  # noqa: E402  (the HIP engine; raises if the library is missing)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
FP32_PEAK_TFLOPS = 157.3  # MI355X packed FP32 (v_pk_fma_f32) dense peak (MI355X_MICROARCH.md)
METRIC = "Msamples/s through WBFM demod chain (NCO+decim+FM discrim) at 1/2/4/8 MI355X"
OFFSETS = [1.5e6, -2.25e6, 0.75e6, -3.5e6, 2.75e6, -0.5e6, 3.75e6, -1.25e6]
METRICS = {  # the non-default configs name what they measure
    "c1": "Msamples/s through 127-tap FirLowpassIq (1 channel, 2^20 cf32 per pass) per MI355X",
    "c3": "Msamples/s through batched 255-tap decimating FIR (256 channels, M=8) per MI355X",
    "c5": "Msamples/s through SSB product demod (128 channels @ 48 ksps) per MI355X",
    "c5f": "Msamples/s through 127-tap channel FIR + SSB product demod (128 channels @ 48 ksps) per MI355X",
}
KERNELS = {"c1": "k_fir_iq8", "c2": "k_wbfm_seg", "c3": "k_decim_w4q", "c4": "k_wbfm_seg", "c5": "k_lpdc_sp",
           "c5f": "k_fir_iq8"}
CHANNELS_PER_GPU = {"c3": 256, "c4": 8, "c5": 128, "c5f": 128}
C3_DESIGN = (10e6, 8, 190e3, 39370.0)  # BASELINE C3: 255 taps (SURVEY §8(d)'s 200e3 cutoff gives 251)
C5F_FIR = (127, 3000.0 / 48e3, 60.0)  # FirLowpassIq::design: +-3 kHz around the SSB channel, 60 dB
NOISE = ("complex AWGN from splitmix64(seed, sample index) + Box-Muller: every sample a function of its "
         "index, so a time shard with its halo is the stream's slice (the reference's add_awgn "
         "sequence, seed 0x1234_5678_ABCD_EF00, cannot be cut that way)")


_M64 = (1 << 64) - 1


def _s64(v):
    """An unsigned 64-bit constant as the int64 with the same bits."""
    v &= _M64
    return v - (1 << 64) if v >> 63 else v


def _srl(z, k):
    """Logical right shift of an int64 tensor."""
    return (z >> k) & ((1 << (64 - k)) - 1)


def index_noise(idx, seed):
    """Complex Gaussian noise (E|w|^2 = 1) as a pure function of the absolute sample
    index: splitmix64 of (seed, index) -> two 24-bit uniforms -> Box-Muller. Any slice
    of a stream gets the same samples whichever rank generates it, so the time shards
    of --shard stream (halos included) are one stream's data."""
    z = idx * _s64(0x9E3779B97F4A7C15) + _s64(seed * 0xD1B54A32D192ED03)
    z = (z ^ _srl(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ _srl(z, 27)) * _s64(0x94D049BB133111EB)
    z = z ^ _srl(z, 31)
    u1 = (_srl(z, 40) + 1).to(torch.float64) * 2.0 ** -24  # (0, 1]
    u2 = (z & 0xFFFFFF).to(torch.float64) * 2.0 ** -24
    del z
    r = torch.sqrt(-torch.log(u1))  # sqrt(-2 ln u1) / sqrt(2): unit power over re + im
    return torch.polar(r, 2 * np.pi * u2).to(torch.complex64)


def wbfm_iq(n, f_off, dev, seed, fs=10e6, t0=0, noise=0.0025):
    """C2 synthetic IQ generated on the device: FM (dev 75 kHz) of
    0.5 sin(1 kHz) + 0.3 sin(7 kHz) at +f_off, plus complex AWGN (P = 0.0025).
    t0: index of the first sample within the stream. Every sample is a function of its
    absolute index alone (the FM phase sum_{j <= k} in closed form, the noise by
    index_noise), so a time shard, halo included, is bit for bit the stream's slice."""
    idx = torch.arange(n, device=dev, dtype=torch.int64) + t0
    kk = (idx + 1).to(torch.float64)  # samples summed into the phase of sample idx

    def sum_sin(w):  # sum_{j < K} sin(w j), closed form
        return torch.sin(w * (kk - 1) / 2) * torch.sin(w * kk / 2) / np.sin(w / 2)

    kdev = 2 * np.pi * 75e3 / fs
    ph = kdev * (0.5 * sum_sin(2 * np.pi * 1e3 / fs) + 0.3 * sum_sin(2 * np.pi * 7e3 / fs))
    del kk
    ph += (2 * np.pi * f_off / fs) * idx.to(torch.float64)
    x = torch.polar(torch.ones_like(ph), ph).to(torch.complex64)
    del ph
    if noise > 0:
        x += index_noise(idx, seed) * np.float32(np.sqrt(noise))
    return x


def channel_plan(cfg, rank, world):
    """The independent channels rank `rank` of `world` owns: [(param, seed)] with
    param the tuning offset (Hz) for C2/C4 and the global channel index for C3/C5.
    Contiguous channel ranges per rank, disjoint, fixed per-rank work (weak
    scaling: C3 256, C4 8, C5 128 channels per GPU; C5's 1024 channels on 8 GPUs);
    nothing on the data path crosses ranks. Every channel's input is
    generated from its own seed, so a channel's output does not depend on the
    rank that runs it."""
    if cfg == "c2":
        return [(OFFSETS[rank % len(OFFSETS)], 0x1234 + rank)]
    if cfg == "c4":
        nch = CHANNELS_PER_GPU["c4"]
        return [(OFFSETS[(rank * nch + c) % len(OFFSETS)] * (1 + 0.01 * c), 0x1234 + rank * nch + c)
                for c in range(nch)]
    if cfg in ("c3", "c5", "c5f"):
        nch = CHANNELS_PER_GPU[cfg]
        base = 77 if cfg == "c3" else 99
        return [(rank * nch + c, (base << 20) ^ (rank * nch + c)) for c in range(nch)]
    raise ValueError(cfg)


_SSB_TONE = {}


def ssb_tone(n, dev):
    """SsbPhasingMod(48e3, 2800, 1500, 0, usb) of a 1.2 kHz tone (0.5
    peak), on the device (the engine's own modulator, the reference's recurrences)."""
    key = (n, str(dev))
    if key not in _SSB_TONE:
        a = (0.5 * torch.sin(2 * np.pi * 1200.0 * torch.arange(n, device=dev, dtype=torch.float64) / 48e3)).float()
        _SSB_TONE[key] = orion_sdr.SsbPhasingMod(48e3, 2800.0, 1500.0).process_device(a.contiguous()).clone()
    return _SSB_TONE[key]


def channel_input(cfg, n, seed, dev):
    """One C3 / C5 channel's synthetic input (complex64, on `dev`), from its seed: C3
    unit-power complex noise; C5 the SSB tone plus AWGN (P = 1e-3) of its own seed."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    if cfg == "c3":
        return torch.randn(n, dtype=torch.complex64, device=dev, generator=g)
    w = torch.randn(n, dtype=torch.complex64, device=dev, generator=g)
    return (ssb_tone(n, dev) + np.float32(np.sqrt(1e-3)) * w).contiguous()


def c1_input(n, dev, seed=0x1234_5678):
    """C1: complex tone at 0.03 fs plus complex noise of power 0.01."""
    t = torch.arange(n, device=dev, dtype=torch.float64)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    x = torch.polar(torch.ones_like(t), 2 * np.pi * 0.03 * t).to(torch.complex64)
    return (x + np.sqrt(0.01) * torch.randn(n, dtype=torch.complex64, device=dev, generator=g)).contiguous()


def max_over_ranks(elapsed, dist, device):
    """Whole-job time: the slowest rank's (the driver's contract). The gloo backend
    reduces host tensors, nccl (RCCL) device tensors."""
    if dist is None:
        return elapsed
    dv = device if dist.get_backend() == "nccl" else torch.device("cpu")
    tt = torch.tensor([elapsed], dtype=torch.float64, device=dv)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def check_shards(x, desc, dist, world, rank, dev):
    """--check-shards (C2 stream shards): each rank runs a FRESH chain, sought to its halo
    start, over its input (the timed handle has run the same samples many times), and
    its audio for [start, stop) is gathered to rank 0 (host tensors over the process
    group), concatenated in rank order and compared with ONE call of a fresh chain over
    the whole stream (generated by the same index-addressed function). Returns the
    comparison on rank 0, None elsewhere."""
    sh = desc["shard"]
    m = 8
    y = orion_sdr.WbfmChain(f_off=OFFSETS[0]).seek(sh["halo_start"]).process_device(x)
    mine = y[(sh["start"] - sh["halo_start"]) // m:].float().cpu()
    parts = [torch.empty(0)] * world
    if dist is not None:
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([mine.numel()], dtype=torch.int64))
        mx = int(max(s.item() for s in sizes))
        buf = torch.zeros(mx)
        buf[: mine.numel()] = mine
        got = [torch.zeros(mx) for _ in range(world)]
        dist.all_gather(got, buf)
        parts = [g[: int(s.item())] for g, s in zip(got, sizes)]
    else:
        parts = [mine]
    if rank != 0:
        return None
    cat = torch.cat(parts).numpy()
    n_all = desc["stream_samples"]
    full = orion_sdr.WbfmChain(f_off=OFFSETS[0]).process_device(
        wbfm_iq(n_all, OFFSETS[0], dev, 0x1234)).cpu().numpy()
    err = float(np.sqrt(np.mean((cat.astype(np.float64) - full) ** 2)) / np.sqrt(np.mean(full.astype(np.float64) ** 2)))
    return {"ranks": world, "stream_samples": n_all, "audio_samples": int(cat.size),
            "one_call_samples": int(full.size), "nrmse_vs_one_call": err,
            "ok": bool(cat.size == full.size and err <= 1e-5)}


def make_workload(cfg, rank, dev, n_override=None, world=1, shard="stream"):
    """Returns (block, x, samples_per_step, bytes_per_sample, description).
    C2 on several ranks: shard="stream" cuts ONE stream of world x n samples in
    time (rank r runs [start, stop) from a STREAM_HALO-sample halo,
    sought to the halo start); shard="channels" gives each rank its own channel."""
    if cfg == "c2" and world > 1 and shard == "stream":
        n = n_override or (1 << 26)
        start, stop, h = orion_sdr.stream_shard(world * n, rank, world)
        blk = orion_sdr.WbfmChain(f_off=OFFSETS[0]).seek(h)
        x = wbfm_iq(stop - h, OFFSETS[0], dev, 0x1234, t0=h)  # one stream: the same seed on every rank
        desc = dict(workload="C2 WBFM chain on ONE stream cut in time: Rotator(-f_off) -> FirDecimator(10e6, 8, "
                    "200e3, 79e3; 127 taps) -> FmQuadratureDemod(1.25e6, 75e3, 15e3) -> FirLowpass(1.25e6, 15e3, "
                    "10e3; 125 taps)", fs_hz=10e6, stream_samples=world * n, samples_per_step_per_gpu=stop - start,
                    halo_samples=start - h, channels_per_gpu=1, noise=NOISE,
                    shard=dict(start=start, stop=stop, halo_start=h))
        return blk, x, stop - start, 8.5, desc
    if cfg == "c2":
        n = n_override or (1 << 26)
        (f_off, seed), = channel_plan(cfg, rank, world)
        blk = orion_sdr.WbfmChain(f_off=f_off)
        x = wbfm_iq(n, f_off, dev, seed)
        desc = dict(workload="C2 WBFM chain: Rotator(-f_off) -> FirDecimator(10e6, 8, 200e3, 79e3; 127 taps) -> "
                    "FmQuadratureDemod(1.25e6, 75e3, 15e3) -> FirLowpass(1.25e6, 15e3, 10e3; 125 taps)",
                    fs_hz=10e6, samples_per_step_per_gpu=n, channels_per_gpu=1, noise=NOISE)
        return blk, x, n, 8.5, desc
    if cfg == "c4":
        plan = channel_plan(cfg, rank, world)
        nch, n = len(plan), n_override or (1 << 24)
        blk = orion_sdr.WbfmChain(f_off=[f for f, _ in plan])
        x = torch.stack([wbfm_iq(n, f, dev, seed) for f, seed in plan]).contiguous()
        desc = dict(workload="C4 WBFM chain, 8 independent channels per GPU", samples_per_step_per_gpu=nch * n,
                    channels_per_gpu=nch, noise=NOISE)
        return blk, x, nch * n, 8.5, desc
    if cfg == "c1":
        n = n_override or (1 << 20)
        blk = orion_sdr.FirLowpassIq.design(127, 0.2, 60.0)
        x = c1_input(n, dev)
        desc = dict(workload="C1 FirLowpassIq::design(127, 0.2, 60 dB) over 2^20 cf32 per pass (the reference's "
                    "CPU Block-graph config, here on the device path)", samples_per_step_per_gpu=n, channels_per_gpu=1,
                    flop_per_sample=508)
        return blk, x, n, 16.0, desc
    if cfg == "c3":
        plan = channel_plan(cfg, rank, world)
        nch, n = len(plan), n_override or (1 << 20)
        blk = orion_sdr.FirDecimator(*C3_DESIGN, channels=nch)
        x = torch.stack([channel_input(cfg, n, seed, dev) for _, seed in plan]).contiguous()
        desc = dict(workload="C3 batched FirDecimator(10e6, 8, 190e3, 39370), 256 channels x 255 taps, M=8",
                    samples_per_step_per_gpu=nch * n, channels_per_gpu=nch, channels=[plan[0][0], plan[-1][0] + 1],
                    input="unit-power complex Gaussian noise per channel (torch generator, seed per channel)")
        return blk, x, nch * n, 9.0, desc
    if cfg == "c5":
        plan = channel_plan(cfg, rank, world)
        nch, n = len(plan), n_override or (1 << 20)
        blk = orion_sdr.SsbProductDemod(48e3, 1500.0, 2800.0, channels=nch)
        x = torch.stack([channel_input(cfg, n, seed, dev) for _, seed in plan]).contiguous()
        desc = dict(workload="C5 SsbProductDemod(48e3, 1500, 2800), 128 channels per GPU @ 48 ksps (1024 on 8 GPUs)",
                    samples_per_step_per_gpu=nch * n, channels_per_gpu=nch, channels=[plan[0][0], plan[-1][0] + 1],
                    input="SsbPhasingMod(48e3, 2800, 1500, 0, usb) of a 1.2 kHz tone (on the device) + AWGN P=1e-3 "
                          "per channel")
        return blk, x, nch * n, 12.0, desc
    if cfg == "c5f":
        plan = channel_plan(cfg, rank, world)
        nch, n = len(plan), n_override or (1 << 20)
        blk = SsbChannelGraph(nch, dev)
        x = torch.stack([channel_input(cfg, n, seed, dev) for _, seed in plan]).contiguous()
        desc = dict(workload="C5 with its channel filter: FirLowpassIq::design(127, 3000/48000, 60 dB) -> "
                    "SsbProductDemod(48e3, 1500, 2800), 128 channels per GPU @ 48 ksps, a two-block device graph "
                    "(the filtered IQ through HBM)", samples_per_step_per_gpu=nch * n, channels_per_gpu=nch,
                    channels=[plan[0][0], plan[-1][0] + 1], flop_per_sample=4 * C5F_FIR[0],
                    input="SsbPhasingMod(48e3, 2800, 1500, 0, usb) of a 1.2 kHz tone (on the device) + AWGN P=1e-3 "
                          "per channel")
        return blk, x, nch * n, 28.0, desc
    raise SystemExit(f"unknown --config {cfg}")


class SsbChannelGraph:
    """C5F: the batched channel filter then the batched SSB demodulator on the device,
    the filtered IQ in an HBM buffer between them (two launches per step). The same
    process_device / out_len surface as a block, for the bench loop."""

    def __init__(self, nch, dev):
        self.fir = orion_sdr.FirLowpassIq.design(*C5F_FIR, channels=nch)
        self.ssb = orion_sdr.SsbProductDemod(48e3, 1500.0, 2800.0, channels=nch)
        self.mid = None
        self.dev = dev

    def out_len(self, n):
        return n

    def process_device(self, x, out=None, stream=None):
        if self.mid is None or self.mid.shape != x.shape:
            self.mid = torch.empty_like(x)
        self.fir.process_device(x, self.mid, stream)
        return self.ssb.process_device(self.mid, out, stream)


def cpu_baseline_channels(x_dev, cfg, seconds_target, f_offs=None):
    """Multi-channel configs: the scalar oracle on min(channels, 16) host threads
    (the oracle's own std::thread pool, channels split over the threads; ctypes
    releases the GIL), over every channel of the step, on a prefix of each sized
    to about `seconds_target` of CPU time (the whole step, repeated, when it is
    shorter than that)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    nch, n_all = x_dev.shape
    thr = max(1, min(nch, 16, os.cpu_count() or 1))
    if cfg == "c3":
        run, what = (lambda xh: O.decim_channels(xh, *C3_DESIGN, thr)), "o_run_decim_channels"
    elif cfg == "c5f":
        taps = O.kaiser_lowpass_taps(*C5F_FIR)

        def run(xh):
            f = np.stack([O.fir_lowpass_iq(xh[c], taps) for c in range(xh.shape[0])])
            return O.ssb_demod_channels(f, 48e3, 1500.0, 2800.0, thr)
        what = "o_fir_lowpass_iq (1 thread) + o_run_ssb_demod_channels"
    elif cfg == "c4":
        run, what = (lambda xh: O.wbfm_channels(xh, np.asarray(f_offs, np.float32), thr)), "o_run_wbfm_channels"
    else:
        run, what = (lambda xh: O.ssb_demod_channels(xh, 48e3, 1500.0, 2800.0, thr)), "o_run_ssb_demod_channels"
    probe = min(n_all, 1 << 14)
    xh = x_dev[:, :probe].cpu().numpy()
    t0 = time.perf_counter()
    run(xh)
    rate = nch * probe / (time.perf_counter() - t0)  # samples per second over all threads
    n = int(min(n_all, max(probe, rate * seconds_target / nch)))
    n -= n % 8
    reps = max(1, int(rate * seconds_target / (nch * n))) if n == n_all else 1
    xh = x_dev[:, :n].cpu().numpy()
    t0 = time.perf_counter()
    for _ in range(reps):
        run(xh)
    dt = time.perf_counter() - t0
    return dict(value=round(reps * nch * n / dt / 1e6, 4), unit="Msamples/s", cores=thr, kind="port",
                sample=f"first {n} samples of all {nch} channels of the rank-0 {cfg.upper()} input"
                       f"{f' (the whole step, {reps} calls)' if reps > 1 or n == n_all else ''}, oracle/orion_oracle.c "
                       f"{what}, {thr} threads, {os.uname().nodename}",
                seconds=round(dt, 2))


def cpu_baseline(x_dev, cfg, seconds_target, max_samples):
    """Scalar oracle ("port") on this host, 1 thread, bounded prefix of the input."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    if cfg == "c1":
        taps = O.kaiser_lowpass_taps(127, 0.2, 60.0)
        n_all = x_dev.shape[-1]
        xh_all = x_dev.cpu().numpy()
        probe = min(n_all, 1 << 16)
        t0 = time.perf_counter()
        O.fir_lowpass_iq(xh_all[:probe], taps)
        rate = probe / (time.perf_counter() - t0)
        passes = max(1, int(rate * seconds_target / n_all))
        t0 = time.perf_counter()
        for _ in range(passes):
            ref = O.fir_lowpass_iq(xh_all, taps)
        dt = time.perf_counter() - t0
        return dict(value=round(passes * n_all / dt / 1e6, 4), unit="Msamples/s", cores=1, kind="port",
                    sample=f"{passes} passes over the whole 2^{np.log2(n_all):.0f}-sample C1 input, oracle/orion_oracle.c "
                           f"o_fir_lowpass_iq, 1 thread, {os.uname().nodename}",
                    seconds=round(dt, 2)), xh_all, ref
    if cfg not in ("c2",):
        return None
    n = min(max_samples, x_dev.shape[-1])
    xh = x_dev[:n].cpu().numpy()
    probe = 1 << 18
    t0 = time.perf_counter()
    O.wbfm(xh[:probe], f_off=OFFSETS[0])
    rate = probe / (time.perf_counter() - t0)
    n = int(min(n, max(probe, rate * seconds_target)))
    n -= n % 8
    t0 = time.perf_counter()
    ref = O.wbfm(xh[:n], f_off=OFFSETS[0])
    dt = time.perf_counter() - t0
    return dict(value=round(n / dt / 1e6, 4), unit="Msamples/s", cores=1, kind="port",
                sample=f"first {n} samples (2^{np.log2(n):.2f}) of the rank-0 C2 input, oracle/orion_oracle.c "
                       f"o_run_wbfm, one call, 1 thread, {os.uname().nodename}",
                seconds=round(dt, 2)), xh[:n], ref


def host_fed(x_dev, passes=3):
    """SURVEY §8(d)'s second figure: the C2 chain fed from HOST memory through the
    path a host caller takes (orion_block_process: Block::process on host slices,
    core.rs:12-22). The same rank-0 input, copied to (a) pinned host memory
    (orion_host_alloc: DMA straight from it) and (b) ordinary pageable memory (the
    handle's pinned staging, CPU copies overlapping the DMA); a fresh chain handle,
    `passes` timed calls each after one warm-up call. Beside them the box's raw
    pinned H2D rate for the same bytes (hipMemcpy through torch's copy_), and the
    fraction of it the pinned path reaches (8 B in per sample)."""
    n = x_dev.shape[-1]
    pin = orion_sdr.pinned_empty((n,), np.complex64)
    pin[:] = x_dev.cpu().numpy()
    res = {}
    for mode, src in (("pinned", pin), ("pageable", None)):
        if src is None:
            src = np.array(pin, copy=True)
        blk = orion_sdr.WbfmChain(f_off=OFFSETS[0])
        out = (orion_sdr.pinned_empty((blk.out_len(n),), np.float32) if mode == "pinned"
               else np.empty(blk.out_len(n), np.float32))
        blk.process_into(src, out)
        t0 = time.perf_counter()
        for _ in range(passes):
            blk.process_into(src, out)
        dt = time.perf_counter() - t0
        res[mode] = passes * n / dt / 1e6
        del src, out, blk
    dst = torch.empty_like(x_dev)
    src_t = torch.from_numpy(pin)
    torch.cuda.synchronize()
    dst.copy_(src_t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(passes):
        dst.copy_(src_t)
    torch.cuda.synchronize()
    h2d = passes * n * 8 / (time.perf_counter() - t0) / 1e9
    del dst, src_t, pin
    return {"value": round(res["pinned"], 2), "unit": "Msamples/s", "input": "pinned host memory (orion_host_alloc)",
            "pageable_value": round(res["pageable"], 2), "h2d_gbs_measured": round(h2d, 2),
            "frac_of_h2d": round(res["pinned"] * 8e6 / (h2d * 1e9), 4), "passes": passes,
            "path": "orion_block_process (host buffers): upload, one device call, download; bytes 8 B in + 0.5 B out "
                    "per sample"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "c5f"])
    ap.add_argument("--n", "--samples", dest="n", type=int, default=0,
                    help="override samples per channel (under torch.distributed.run use --samples: its own "
                         "parser reads --n as an abbreviation of its options)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-max-samples", type=int, default=1 << 24)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-h2d", action="store_true", help="skip the host-fed (H2D-inclusive) C2 figure")
    ap.add_argument("--rest", type=float, default=0.0, help="idle seconds between input synthesis and the warm-up")
    ap.add_argument("--shard", default="stream", choices=["stream", "channels"],
                    help="C2 on several GPUs: one stream cut in time (with a halo), or a channel per GPU")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for the timing barrier / max (nccl = RCCL; gloo: host tensors, "
                         "several ranks may share a device)")
    ap.add_argument("--device-map", default="",
                    help="comma list: the device of each local rank (default: local rank i on device i)")
    ap.add_argument("--check-shards", action="store_true",
                    help="C2 stream shards: gather the ranks' audio and compare with one call over the stream")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.gpus != world:  # one process per GPU: N > 1 needs the launcher (torch.distributed.run)
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N > 1 as "
                         f"python -m torch.distributed.run --nproc-per-node N bench.py --gpus N")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dmap = [int(v) for v in args.device_map.split(",")] if args.device_map else None
    if dmap is not None and len(dmap) <= local:
        raise SystemExit(f"bench.py: --device-map {args.device_map} has no entry for local rank {local}")
    gpu = dmap[local] if dmap is not None else local
    if args.dist_backend == "nccl" and dmap is not None and len(set(dmap)) != len(dmap):
        raise SystemExit("bench.py: ranks sharing a device need --dist-backend gloo (RCCL wants one rank per GPU)")
    dist = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    stream = torch.cuda.current_stream(dev)

    blk, x, samples, bps, desc = make_workload(args.config, rank, dev, args.n or None, world, args.shard)
    nout = blk.out_len(x.shape[-1])
    out_shape = (nout,) if x.dim() == 1 else (x.shape[0], nout)
    out_dtype = torch.complex64 if args.config in ("c1", "c3") else torch.float32
    if args.check_shards and "shard" not in desc:
        raise SystemExit("bench.py: --check-shards needs --config c2 on several ranks with --shard stream")
    out = torch.empty(out_shape, dtype=out_dtype, device=dev)
    torch.cuda.synchronize(dev)
    if args.rest > 0:
        time.sleep(args.rest)

    def step():
        blk.process_device(x, out, stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    # kernel timing: one pair of HIP events on the launch stream brackets the K
    # back-to-back launches (per-step events would add their own packets between
    # the kernels); the average includes the inter-launch gaps (conservative)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dist, dev)
    kern_ms = ev0.elapsed_time(ev1) / args.steps

    total = samples * world * args.steps
    value = total / elapsed / 1e6
    achieved = samples * bps / (kern_ms * 1e-3) / 1e9  # GB/s, one launch per step
    line = {
        "metric": METRICS.get(args.config, METRIC), "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        **({"audio_fir": "f16 hi+lo MFMA (v_mfma_f32_16x16x32_f16, per-sub-range scale), f32 accumulate"}
           if args.config in ("c2", "c4") else {}),
        "config": dict(desc, parallelism=(f"stream time-sharded x{world} (halo {orion_sdr.STREAM_HALO} samples), no "
                                          "data-path collective" if "halo_samples" in desc
                                          else f"channel-sharded x{world}, no data-path collective"),
                       **({"dist_backend": args.dist_backend} if world > 1 else {}),
                       **({"device_map": args.device_map} if dmap is not None else {})),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": KERNELS[args.config],
                     "kernel_ms": round(kern_ms, 4), "bytes_per_sample": bps},
        "cpu_baseline": None,
    }
    if args.config == "c5f":
        # the dominant kernel alone (the 127-tap FIR, FP32-bound: 508 flop per sample), one
        # event pair around each FIR launch after the timed region; the SSB scan beside it
        mid = torch.empty_like(x)
        fe, se = [], []
        for _ in range(max(args.steps, 10)):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(stream)
            blk.fir.process_device(x, mid, stream.cuda_stream)
            e1.record(stream)
            blk.ssb.process_device(mid, out, stream.cuda_stream)
            e2.record(stream)
            fe.append((e0, e1))
            se.append((e1, e2))
        torch.cuda.synchronize(dev)
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in fe]))
        ssb_ms = float(np.mean([a.elapsed_time(b) for a, b in se]))
        line["roofline"]["kernel_ms"] = round(kern_ms, 4)
        line["roofline"]["second_kernel"] = {"kernel": "k_lpdc_sp", "kernel_ms": round(ssb_ms, 4),
                                             "hbm_gbs": round(samples * 12.0 / (ssb_ms * 1e-3) / 1e9, 1)}
        del mid
    if args.config in ("c1", "c5f"):  # compute-bound: packed FP32 is the roof (31.75 flop/B > the ~19.7 flop/B ridge)
        achieved = samples * 16.0 / (kern_ms * 1e-3) / 1e9  # the FIR's own bytes: 8 B in + 8 B out
        tflops = samples * desc["flop_per_sample"] / (kern_ms * 1e-3) / 1e12
        line["roofline"].update(bound="fp32", achieved=round(tflops, 2), peak=FP32_PEAK_TFLOPS, unit="TFLOP/s",
                                frac=round(tflops / FP32_PEAK_TFLOPS, 4), hbm_gbs=round(achieved, 1),
                                hbm_frac=round(achieved / HBM_PEAK_GBS, 4))
    # per-launch spread (after the timed region): one event pair per launch,
    # so the clock's step-down across back-to-back launches is visible beside the average
    pairs = []
    for _ in range(max(args.steps, 10)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        step()
        e1.record(stream)
        pairs.append((e0, e1))
    torch.cuda.synchronize(dev)
    per = sorted(e0.elapsed_time(e1) for e0, e1 in pairs)
    line["roofline"]["per_launch_ms"] = {"min": round(per[0], 4), "median": round(per[len(per) // 2], 4),
                                         "max": round(per[-1], 4), "launches": len(per)}
    # on-box read ceiling (after the timed region): the library's streaming-read probe
    # over this rank's input, 10 launches between events. Diagnostic
    # only: a probe that cannot run (input below one tile per wave) leaves it null.
    try:
        nb = orion_sdr.diag_stream_read(x, stream.cuda_stream) if args.config != "c1" else 0
        if nb > 0:
            p0, p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            p0.record(stream)
            for _ in range(10):
                orion_sdr.diag_stream_read(x, stream.cuda_stream)
            p1.record(stream)
            torch.cuda.synchronize(dev)
            peak_meas = nb / (p0.elapsed_time(p1) / 10 * 1e-3) / 1e9
            line["roofline"]["peak_measured"] = round(peak_meas, 1)
            line["roofline"]["frac_measured"] = round(achieved / peak_meas, 4)
    except Exception as e:  # noqa: BLE001  (the bench line must still print)
        line["roofline"]["peak_measured"] = None
        line["roofline"]["probe_error"] = str(e)[:120]
    # PMC traffic is collected in separate rocprofv3 --pmc passes (tools/traffic.py), never
    # inside this run: the figure is the committed file's, and the line names it
    traffic_file = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(traffic_file):
        tr = json.load(open(traffic_file))
        if tr.get("samples_per_launch") == samples:
            line["roofline"]["traffic"] = tr.get("hbm_bytes_per_launch")
            line["roofline"]["traffic_source"] = f"profiles/traffic_{args.config}.json (rocprofv3 --pmc FETCH_SIZE + " \
                                                 f"WRITE_SIZE, separate passes; not measured in this run)"
    if args.check_shards:
        line["shard_check"] = check_shards(x, desc, dist, world, rank, dev)
    if rank == 0 and world == 1 and args.config == "c2" and not args.no_h2d:
        try:
            line["host_fed"] = host_fed(x)
        except Exception as e:  # noqa: BLE001  (the bench line must still print)
            line["host_fed"] = {"error": str(e)[:160]}
    if rank == 0 and world == 1 and not args.no_cpu and args.config in ("c1", "c2"):
        res = cpu_baseline(x, args.config, args.cpu_seconds, args.cpu_max_samples)
        if res:
            cb, xh, ref = res
            fresh = (orion_sdr.WbfmChain(f_off=OFFSETS[0]) if args.config == "c2"
                     else orion_sdr.FirLowpassIq.design(127, 0.2, 60.0))
            got = fresh.process(xh)
            den = float(np.sqrt(np.mean(np.abs(ref.astype(np.complex128)) ** 2)))
            cb["gpu_vs_cpu_nrmse"] = float(np.sqrt(np.mean(np.abs(got.astype(np.complex128) - ref) ** 2)) / den)
            line["cpu_baseline"] = cb
    elif rank == 0 and world == 1 and not args.no_cpu:
        f_offs = [f for f, _ in channel_plan("c4", 0, 1)] if args.config == "c4" else None
        line["cpu_baseline"] = cpu_baseline_channels(x, args.config, min(args.cpu_seconds, 10.0), f_offs)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
