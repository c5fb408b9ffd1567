import sys, torch, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'orion-sdr_amd')
import bench, orion_sdr
dev = torch.device('cuda', 0)
n = 1 << 22
outs = []
for r in range(2):
    blk, x, s, b, d = bench.make_workload('c2', r, dev, n, 2, 'stream')
    out = torch.empty(blk.out_len(x.shape[-1]), dtype=torch.float32, device=dev)
    blk.process_device(x, out, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    start, stop, h = orion_sdr.stream_shard(2 * n, r, 2)
    outs.append(out[(start - h) // 8:].cpu().numpy())
    print(r, s, d['halo_samples'], x.shape)
# reference: the whole stream (noise differs per rank slice, so compare against a
# single handle over the concatenated rank inputs)
xs = []
for r in range(2):
    start, stop, h = orion_sdr.stream_shard(2 * n, r, 2)
    xs.append(bench.wbfm_iq(stop - h, bench.OFFSETS[0], dev, 0x1234 + r, t0=h)[start - h:])
xf = torch.cat(xs)
full = orion_sdr.WbfmChain(f_off=bench.OFFSETS[0])
of = torch.empty(full.out_len(xf.shape[-1]), dtype=torch.float32, device=dev)
full.process_device(xf, of, torch.cuda.current_stream(dev).cuda_stream)
torch.cuda.synchronize()
got = np.concatenate(outs); ref = of.cpu().numpy()
# rank 1's halo comes from its own (differently seeded) slice, so compare away from the cut
cut = n // 8
e = np.abs(got - ref); rms = np.sqrt(np.mean(ref ** 2))
print("len", len(got), len(ref), "nrmse rank0", np.sqrt(np.mean(e[:cut] ** 2)) / rms,
      "nrmse rank1 after 2048", np.sqrt(np.mean(e[cut + 2048:] ** 2)) / rms)
