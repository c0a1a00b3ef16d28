"""Parity at the north-star size (BASELINE.json: 1 M x 4 KiB masked TEXT frames, 1 GPU),
through size-independent properties the oracle does not need to replay:
  * unmasking is an involution: every decoded payload XOR its frame's mask is the wire
    payload, checked over all 4.3 GB on the device;
  * UTF-8 verdicts: invalid bytes planted in chosen frames fail exactly those sessions at
    exactly those frames with the reference's 1007 error, every other session delivers
    all its frames."""
import pytest

pytestmark = pytest.mark.gpu

F, P, S = 1 << 20, 4096, 1024
FLEN = P + 8  # 2 + 2 (u16 length) + 4 (mask)


@pytest.fixture(scope="module")
def batch():
    import torch
    from snf4j_amd import Context
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    wire = torch.empty(F * FLEN + 64, dtype=torch.uint8, device=dev)
    off = torch.empty(F + 1, dtype=torch.int64, device=dev)
    sf = torch.empty(S + 1, dtype=torch.int32, device=dev)
    ctx.synth_uniform(0x5EED, F, P, F // S, 1, True, 1, wire, off, sf)
    yield ctx, dev, wire, off, sf
    ctx.close()


def _decode(ctx, dev, wire, off, sf):
    import torch
    from snf4j_amd import decoder_cfg
    payload = torch.empty(F * FLEN + 16 * F + 16, dtype=torch.uint8, device=dev)
    desc = torch.empty(F * 16, dtype=torch.uint8, device=dev)
    res = torch.empty(S * 16, dtype=torch.uint8, device=dev)
    state = torch.zeros(S * 8, dtype=torch.uint8, device=dev)
    ctx.decode_device(decoder_cfg(False, False, 65536, True), wire, off, sf, state, payload, desc, res,
                      wire_len=F * FLEN)
    torch.cuda.synchronize(dev)
    return payload, desc, res


def test_full_size_unmask_involution(batch):
    import numpy as np
    import torch
    from snf4j_amd._lib import DESC_DTYPE, RESULT_DTYPE
    ctx, dev, wire, off, sf = batch
    payload, desc, res = _decode(ctx, dev, wire, off, sf)
    r = res.cpu().numpy().view(RESULT_DTYPE)
    assert int(r["error"].max()) == 0 and int(r["n_delivered"].sum()) == F
    d = desc.cpu().numpy().view(DESC_DTYPE)
    assert (d["payload_len"] == P).all() and (d["opcode"] == 1).all()
    assert np.array_equal(d["payload_off"], np.arange(F, dtype=np.uint64) * P)  # 4 KiB slots, in order
    w = wire[:F * FLEN].view(F, FLEN)
    for c0 in range(0, F, 1 << 17):  # 128 K frames (0.5 GB) at a time
        c1 = c0 + (1 << 17)
        mask = w[c0:c1, 4:8].repeat(1, P // 4)
        got = payload[c0 * P:c1 * P].view(c1 - c0, P)
        assert torch.equal(got ^ mask, w[c0:c1, 8:]), c0


def test_full_size_planted_utf8_errors(batch):
    import torch
    from snf4j_amd._lib import RESULT_DTYPE
    ctx, dev, wire, off, sf = batch
    fps = F // S
    plant = {3: (17, 0), 500: (1023, 4095), 1023: (0, 2048)}  # session -> (frame in session, payload byte)
    w = wire[:F * FLEN].view(F, FLEN)
    saved = []
    for s, (j, b) in plant.items():
        k = s * fps + j
        saved.append((k, b, int(w[k, 8 + b].item())))
        w[k, 8 + b] = w[k, 4 + (b & 3)] ^ 0xFF  # unmasks to 0xFF: never valid UTF-8
    try:
        _, _, res = _decode(ctx, dev, wire, off, sf)
    finally:
        for k, b, v in saved:
            w[k, 8 + b] = v
    r = res.cpu().numpy().view(RESULT_DTYPE)
    for s in range(S):
        if s in plant:
            assert int(r["error"][s]) == 14 and int(r["close_code"][s]) == 1007, s
            assert int(r["n_delivered"][s]) == plant[s][0], s
        else:
            assert int(r["error"][s]) == 0 and int(r["n_delivered"][s]) == fps, s
