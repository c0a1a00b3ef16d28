"""Parity at full size, through size-independent properties the oracle does not need
to replay, on the north-star batch (BASELINE.json: 1 M x 4 KiB masked TEXT frames,
1 GPU) and on configs[3]'s per-GPU shard (64 M x 4 KiB over 8 GPUs = 8 M x 4 KiB,
34.4 GB in + 34.4 GB out in one batch on one GPU):
  * unmasking is an involution: every decoded payload XOR its frame's mask is the wire
    payload, checked over all 4.3 GB on the device;
  * UTF-8 verdicts: invalid bytes planted in chosen frames fail exactly those sessions at
    exactly those frames with the reference's 1007 error, every other session delivers
    all its frames."""
import pytest

import benchsupport

pytestmark = pytest.mark.gpu

P, S = 4096, 1024
FLEN = P + 8  # 2 + 2 (u16 length) + 4 (mask)


@pytest.fixture(scope="module", params=[1 << 20, 8 << 20], ids=["north_1Mx4K", "configs3_shard_8Mx4K"])
def batch(request):
    import torch
    from snf4j_amd import Context
    F = request.param
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    wire = torch.empty(F * FLEN + 64, dtype=torch.uint8, device=dev)
    off = torch.empty(F + 1, dtype=torch.int64, device=dev)
    sf = torch.empty(S + 1, dtype=torch.int32, device=dev)
    benchsupport.synth_uniform(ctx, 0x5EED ^ F, F, P, F // S, 1, True, 1, wire, off, sf)
    yield F, ctx, dev, wire, off, sf
    ctx.close()
    del wire, off, sf
    torch.cuda.empty_cache()


def _decode(F, ctx, dev, wire, off, sf):
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
    F, ctx, dev, wire, off, sf = batch
    payload, desc, res = _decode(F, ctx, dev, wire, off, sf)
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
    F, ctx, dev, wire, off, sf = batch
    fps = F // S
    plant = {3: (17, 0), 500: (fps - 1, 4095), 1023: (0, 2048)}  # session -> (frame in session, payload byte)
    w = wire[:F * FLEN].view(F, FLEN)
    saved = []
    for s, (j, b) in plant.items():
        k = s * fps + j
        saved.append((k, b, int(w[k, 8 + b].item())))
        w[k, 8 + b] = w[k, 4 + (b & 3)] ^ 0xFF  # unmasks to 0xFF: never valid UTF-8
    try:
        _, _, res = _decode(F, ctx, dev, wire, off, sf)
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


def test_full_size_encode_decode_round_trip():
    """configs[4] at full size: 64 x 16 MiB messages in 64 KiB frames, client-masked on the
    GPU, then decoded by the server path on the GPU: every payload byte comes back, every
    header is the reference's (BINARY then CONTINUATION, FIN on the last, u64 length form)."""
    import numpy as np
    import torch
    from snf4j_amd import Context, decoder_cfg, encoded_length
    from snf4j_amd._lib import DESC_DTYPE, ENCODE_DTYPE, RESULT_DTYPE
    M, FR, FP = 64, 256, 65536
    n = M * FR
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    try:
        g = torch.Generator(device=dev).manual_seed(9)
        payload = torch.randint(0, 256, (n * FP,), dtype=torch.uint8, device=dev, generator=g)
        fr = np.zeros(n, dtype=ENCODE_DTYPE)
        fr["payload_off"] = np.arange(n, dtype=np.uint64) * FP
        fr["payload_len"] = FP
        j = np.arange(n) % FR
        fr["opcode"] = np.where(j == 0, 2, 0)
        fr["flags"] = np.where(j == FR - 1, 0x80, 0)
        fr["mask"] = np.random.default_rng(5).integers(0, 256, (n, 4), dtype=np.uint8)
        frames = torch.from_numpy(fr.view(np.uint8).copy()).to(dev)
        sfe = torch.from_numpy((np.arange(M + 1) * FR).astype(np.int32)).to(dev)
        closed = torch.zeros(M, dtype=torch.uint8, device=dev)
        elen = encoded_length(FP, True)
        wire = torch.empty(n * elen + 64, dtype=torch.uint8, device=dev)
        wire_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        ctx.encode_device(True, payload, frames, sfe, closed, wire, wire_off)
        torch.cuda.synchronize(dev)
        assert int(wire_off[-1].item()) == n * elen
        w = wire[:n * elen].view(n, elen)
        hdr = w[:, :10].cpu().numpy()
        assert (hdr[:, 1] == 0xFF).all() and (hdr[:, 2:10] == np.array([0, 0, 0, 0, 0, 1, 0, 0], np.uint8)).all()
        assert (hdr[:, 0] == np.where(j == 0, 0x02, 0x00) | np.where(j == FR - 1, 0x80, 0)).all()
        assert np.array_equal(w[:, 10:14].cpu().numpy(), fr["mask"])
        out = torch.empty(n * elen + 16 * n + 16, dtype=torch.uint8, device=dev)
        desc = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        res = torch.empty(M * 16, dtype=torch.uint8, device=dev)
        state = torch.zeros(M * 8, dtype=torch.uint8, device=dev)
        ctx.decode_device(decoder_cfg(False, False, 65536, True), wire, wire_off, sfe, state, out, desc, res,
                          wire_len=n * elen)
        torch.cuda.synchronize(dev)
        r = res.cpu().numpy().view(RESULT_DTYPE)
        assert int(r["error"].max()) == 0 and int(r["n_delivered"].sum()) == n
        d = desc.cpu().numpy().view(DESC_DTYPE)
        assert np.array_equal(d["payload_off"], np.arange(n, dtype=np.uint64) * FP)
        assert torch.equal(out[:n * FP], payload)
    finally:
        ctx.close()


def test_configs1_full_size_binary_involution_and_no_errors():
    """configs[1] at full size: 1 M masked BINARY frames of 1 KiB, 256 sessions (the
    unmask-only line; BINARY frames take no UTF-8 check): zero errors, every frame
    delivered in order into 1 KiB slots, and every payload XOR its mask is the wire
    payload, over all 1.07 GB on the device; then planted protocol errors (a reserved
    opcode, a clear mask bit) fail exactly those sessions at exactly those frames."""
    import numpy as np
    import torch
    from snf4j_amd import Context, decoder_cfg
    from snf4j_amd._lib import DESC_DTYPE, RESULT_DTYPE
    F, P1, S1 = 1 << 20, 1024, 256
    FL = P1 + 8
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    try:
        wire = torch.empty(F * FL + 64, dtype=torch.uint8, device=dev)
        off = torch.empty(F + 1, dtype=torch.int64, device=dev)
        sf = torch.empty(S1 + 1, dtype=torch.int32, device=dev)
        benchsupport.synth_uniform(ctx, 0xC0F1, F, P1, F // S1, 2, True, 0, wire, off, sf)

        def decode():
            payload = torch.empty(F * FL + 16 * F + 16, dtype=torch.uint8, device=dev)
            desc = torch.empty(F * 16, dtype=torch.uint8, device=dev)
            res = torch.empty(S1 * 16, dtype=torch.uint8, device=dev)
            state = torch.zeros(S1 * 8, dtype=torch.uint8, device=dev)
            ctx.decode_device(decoder_cfg(False, False, 65536, True), wire, off, sf, state, payload, desc, res,
                              wire_len=F * FL)
            torch.cuda.synchronize(dev)
            return payload, desc.cpu().numpy().view(DESC_DTYPE), res.cpu().numpy().view(RESULT_DTYPE)

        payload, d, r = decode()
        assert int(r["error"].max()) == 0 and (r["n_delivered"] == F // S1).all()
        assert (d["payload_len"] == P1).all() and (d["opcode"] == 2).all() and (d["flags"] & 0x80 == 0x80).all()
        assert np.array_equal(d["payload_off"], np.arange(F, dtype=np.uint64) * P1)
        w = wire[:F * FL].view(F, FL)
        assert (w[:, 0] == 0x82).all() and (w[:, 1] == 0xFE).all()
        for c0 in range(0, F, 1 << 18):
            c1 = c0 + (1 << 18)
            mask = w[c0:c1, 4:8].repeat(1, P1 // 4)
            assert torch.equal(payload[c0 * P1:c1 * P1].view(c1 - c0, P1) ^ mask, w[c0:c1, 8:]), c0
        del payload
        fps = F // S1
        plant = {7: (100, 0x83), 200: (fps - 1, 0x02)}  # session -> (frame, byte 0 / byte 1 change)
        k7, k200 = 7 * fps + 100, 200 * fps + fps - 1
        b0, b1 = int(w[k7, 0].item()), int(w[k200, 1].item())
        w[k7, 0] = 0x83          # reserved opcode 3: "Invalid opcode", 1002
        w[k200, 1] = 0x7E        # mask bit clear from a client: "Masking", 1002
        try:
            _, _, r = decode()
        finally:
            w[k7, 0], w[k200, 1] = b0, b1
        for s in range(S1):
            if s in plant:
                assert int(r["error"][s]) != 0 and int(r["close_code"][s]) == 1002, s
                assert int(r["n_delivered"][s]) == plant[s][0], s
            else:
                assert int(r["error"][s]) == 0 and int(r["n_delivered"][s]) == fps, s
    finally:
        ctx.close()
        torch.cuda.empty_cache()
