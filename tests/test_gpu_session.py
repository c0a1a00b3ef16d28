"""The drop-in decoder as snf4j runs it, on the GPU: GpuFrameDecoder
(java/.../GpuFrameDecoder.java, restated in snf4j_amd/loop.py) inside the restated
stream session read loop (StreamSession.java:765-854, both consume paths, heap and
direct buffers), over the native batcher (DecoderBatcher -> wsg_batcher_* ->
decode kernels), all sessions on one selector loop with flushes in flight.

Every session's handler events and ending — frames (opcode, FIN, RSV, payload), the
exception and its message, writenf(CloseFrame(code)), close() / quickClose() — equal
the reference pipeline's, where "ws-decoder" is the oracle's FrameDecoder
(FrameDecoder.java:92-401 + FrameUtf8Validator.java:59-98) and the session ends as
InternalSession.exception/controlClose says (InternalSession.java:804-848): decoders
behind "ws-decoder" and handlers that throw GENTLE, NONE, DEFAULT and plain
exceptions, protocol errors found by the device, and u64 length errors thrown from
available() (FrameDecoder.java:388-394) after the frames before them arrived."""
import pytest

from tests import sessionmodel as M

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from snf4j_amd import Context
    c = Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_gpu_frame_decoder_sessions_match_reference(ctx, oracle, seed):
    from benchsupport.selector import SelectorLoop
    from snf4j_amd.loop import DecoderBatcher
    plan = M.make_plan(seed, 64)
    want = M.run_reference(oracle, plan)
    loop = SelectorLoop()
    b = DecoderBatcher(loop, len(plan), ctx=ctx, max_wire=4 << 20, max_frames=1 << 14)
    try:
        got = M.run_dropin(plan, b, seed=seed)
    finally:
        b.close()
    for i, (w, g) in enumerate(zip(want, got)):
        assert g == w, (i, plan[i]["dec"], plan[i]["hnd"], w[-4:], g[-4:])
    assert M.endings(want) >= {"GENTLE", "NONE", "DEFAULT", "PLAIN", "InvalidFrameException", "length", "close",
                               "quickClose"}, M.endings(want)
    assert b.stats["flushes"] >= 3, b.stats
