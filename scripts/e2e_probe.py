"""e2e overlap probe: enqueue cost of wsg_decode_batch_host_async, and a 3-stream
(H2D / kernels / D2H) event pipeline with the device API."""
import sys
import time

import torch

sys.path.insert(0, ".")
import benchsupport  # noqa: E402
import snf4j_amd  # noqa: E402

F, P, S = 1 << 18, 4096, 256
dev = torch.device("cuda", 0)
flen = snf4j_amd.encoded_length(P, True)
WB = F * flen
ctx0 = snf4j_amd.Context(0)
wire = torch.empty(WB + 64, dtype=torch.uint8, device=dev)
off = torch.empty(F + 1, dtype=torch.int64, device=dev)
sf = torch.empty(S + 1, dtype=torch.int32, device=dev)
benchsupport.synth_uniform(ctx0, 7, F, P, F // S, 1, True, 1, wire, off, sf)
torch.cuda.synchronize(dev)
cfg = snf4j_amd.decoder_cfg(False, False, 65536, True)
h_wire = wire[:WB].cpu().pin_memory()
h_off, h_sf = off.cpu().pin_memory(), sf.cpu().pin_memory()
PB = WB + 16 * F + 16

# (a) async host API on two contexts: enqueue time per call
streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
ctxs = [snf4j_amd.Context(0, stream=s) for s in streams]
bufs = [dict(pay=torch.empty(PB, dtype=torch.uint8).pin_memory(), desc=torch.empty(F * 16, dtype=torch.uint8).pin_memory(),
             res=torch.empty(S * 16, dtype=torch.uint8).pin_memory(), st=torch.zeros(S * 8, dtype=torch.uint8).pin_memory())
        for _ in range(2)]
for i in range(2):
    b = bufs[i]
    ctxs[i].decode_host_async(cfg, h_wire, h_off, h_sf, b["st"], b["pay"], b["desc"], b["res"])
torch.cuda.synchronize(dev)
reps = 8
enq = []
t0 = time.perf_counter()
for i in range(reps):
    b = bufs[i % 2]
    t1 = time.perf_counter()
    ctxs[i % 2].decode_host_async(cfg, h_wire, h_off, h_sf, b["st"], b["pay"], b["desc"], b["res"])
    enq.append(time.perf_counter() - t1)
torch.cuda.synchronize(dev)
t = (time.perf_counter() - t0) / reps
print(f"async API x2 ctx: {WB / t / 2**30:.1f} GiB/s, {t*1e3:.1f} ms/batch, enqueue ms {[round(e*1e3,1) for e in enq]}")

# (b) 3 streams + events, device API, torch copies
sh, sk, sd = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
ctxk = snf4j_amd.Context(0, stream=sk)
dw = [torch.empty(WB + 64, dtype=torch.uint8, device=dev) for _ in range(2)]
dp = [torch.empty(PB, dtype=torch.uint8, device=dev) for _ in range(2)]
dd = [torch.empty(F * 16, dtype=torch.uint8, device=dev) for _ in range(2)]
dr = [torch.empty(S * 16, dtype=torch.uint8, device=dev) for _ in range(2)]
dst = torch.zeros(S * 8, dtype=torch.uint8, device=dev)
ev_in = [torch.cuda.Event() for _ in range(2)]
ev_k = [torch.cuda.Event() for _ in range(2)]
ev_out = [torch.cuda.Event() for _ in range(2)]
for e in ev_out:
    e.record(sd)


def batch(i):
    j = i % 2
    b = bufs[j]
    sh.wait_event(ev_k[j]) if i >= 2 else None  # device wire buffer j free once its decode is done
    with torch.cuda.stream(sh):
        dw[j][:WB].copy_(h_wire, non_blocking=True)
        ev_in[j].record(sh)
    sk.wait_event(ev_in[j])
    sk.wait_event(ev_out[j])  # payload buffer j free once its D2H is done
    ctxk.decode_device(cfg, dw[j], off, sf, dst, dp[j], dd[j], dr[j], wire_len=WB)
    ev_k[j].record(sk)
    sd.wait_event(ev_k[j])
    with torch.cuda.stream(sd):
        b["pay"].copy_(dp[j], non_blocking=True)
        b["desc"].copy_(dd[j], non_blocking=True)
        ev_out[j].record(sd)


batch(0); batch(1)
torch.cuda.synchronize(dev)
t0 = time.perf_counter()
for i in range(reps):
    batch(i)
torch.cuda.synchronize(dev)
t = (time.perf_counter() - t0) / reps
print(f"3-stream events: {WB / t / 2**30:.1f} GiB/s, {t*1e3:.1f} ms/batch")
