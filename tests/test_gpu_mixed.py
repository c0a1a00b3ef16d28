"""GPU parity on the mixed configuration (BASELINE configs[2]): log-uniform 64 B-64 KiB
text+binary messages, fragmented at arbitrary bytes (code points split across
fragments), injected invalid UTF-8; bytes generated on the device by wsg_synth_frames,
decoded on the device, checked frame by frame against the oracle."""
import numpy as np
import pytest

from tests.test_gpu_decode import compare

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,sessions,mib,bad", [(1, 64, 24, 0.05), (2, 7, 8, 0.0), (3, 256, 32, 0.01)])
def test_mixed_batch_parity(oracle, seed, sessions, mib, bad):
    import torch

    from snf4j_amd import Context, decoder_cfg
    from snf4j_amd._lib import DESC_DTYPE, RESULT_DTYPE, STATE_DTYPE, lib
    from snf4j_amd.synth import mixed_plan

    t, off, sf, wl, info = mixed_plan(seed, sessions, mib << 20, bad_frac=bad, frag_frac=0.2)
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    try:
        tab = torch.from_numpy(t.view(np.uint8).copy()).to(dev)
        wire = torch.zeros(wl + 64, dtype=torch.uint8, device=dev)
        ctx.synth_frames(tab, wire)
        n, n_s = len(t), len(sf) - 1
        cap = int(lib.wsg_decode_payload_bound(wl, n))
        payload = torch.empty(cap, dtype=torch.uint8, device=dev)
        desc = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        res = torch.empty(n_s * 16, dtype=torch.uint8, device=dev)
        state = torch.zeros(n_s * 8, dtype=torch.uint8, device=dev)
        ctx.decode_device(decoder_cfg(False, False, 65536, True), wire, torch.from_numpy(off.astype(np.int64)).to(dev),
                          torch.from_numpy(sf.astype(np.int32)).to(dev), state, payload, desc, res, wire_len=wl)
        torch.cuda.synchronize(dev)
        h_wire = wire[:wl].cpu().numpy()
        gpu = (payload.cpu().numpy(), desc.cpu().numpy().view(DESC_DTYPE), res.cpu().numpy().view(RESULT_DTYPE))
    finally:
        ctx.close()
    ora = oracle.Batch(False, False, 65536, True, n_s).decode(h_wire, off, sf)
    compare(gpu, ora, sf, f"mixed seed {seed}")
    # the generator: exactly the sessions holding an injected sequence fail, with 1007
    err = gpu[2]["error"]
    bad_s = set(info["bad_sessions"])
    for s in range(n_s):
        assert (int(err[s]) == 14) == (s in bad_s), s
        assert int(err[s]) in (0, 14)
