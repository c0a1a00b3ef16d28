"""The restated snf4j read loop and exception path (snf4j_amd/loop.py) on the CPU:

* StreamSession's two consume loops (StreamSession.java:765-854) with the oracle's
  FrameDecoder deliver exactly the oracle's read loop's frames and first error, over
  random socket reads, heap and direct buffers;
* controlClose (InternalSession.java:804-848): GENTLE -> exception(closing cause) +
  close, NONE -> exception only, DEFAULT / any other exception -> quickClose;
* GpuFrameDecoder's host logic (available / checked / decode / deliver / downstream /
  fail, java/.../GpuFrameDecoder.java) run against a CPU batcher (tests/sessionmodel.py
  OracleBatcher) gives every session the same handler events and the same ending as
  the reference pipeline, with decoders and handlers that throw each close type and
  u64 length errors thrown from available().  tests/test_gpu_session.py runs the same
  plans through the native batcher on the GPU."""
import random

import numpy as np
import pytest

from benchsupport.selector import SelectorLoop
from snf4j_amd.loop import CloseType
from tests.harness.session import StreamSession
from tests import sessionmodel as M
from tests import wsgen


@pytest.mark.parametrize("optimized", [False, True])
@pytest.mark.parametrize("direct", [False, True])
def test_consume_loops_match_the_oracle_read_loop(oracle, optimized, direct):
    rng = random.Random(11 + optimized * 2 + direct)
    nrng = np.random.default_rng(11)
    for s in range(40):
        inject = wsgen.INJECT_KINDS[rng.randrange(len(wsgen.INJECT_KINDS))] if s % 4 == 0 else None
        stream = b"".join(wsgen.session_frames(nrng, rng.randrange(1, 12), big=(s % 5 == 0), inject=inject))
        sess = StreamSession([("ws-decoder", M.RefFrameDecoder(oracle))], optimized=optimized, direct=direct)
        pos = 0
        while pos < len(stream) and not sess.closing:
            n = rng.randrange(1, 9000)
            sess.read_event(stream[pos:pos + n])
            pos += n
        frames, err = oracle.stream_decode(stream)
        got = [e[1] for e in sess.events if e[0] == "read"]
        assert [(f.opcode, f.fin, f.rsv, f.payload) for f in frames] == \
               [(int(f.getOpcode()), f.isFinalFragment(), f.getRsvBits(), f.getPayload()) for f in got], s
        exc = [e[1] for e in sess.events if e[0] == "exception"]
        assert [str(x) for x in exc] == ([str(err)] if err else []), s
        if err:  # FrameDecoder: writenf(CloseFrame(code)), then the GENTLE close
            assert [e[0] for e in sess.events[-3:]] == ["writenf", "exception", "close"], s
            assert sess.events[-3][1].getStatus() == err.close_code


def test_control_close_rules():
    s = StreamSession([("ws-decoder", None)])
    g = M.GentleError("g")
    s.exception(g)
    assert s.events == [("exception", g.cause), ("close",)]
    s = StreamSession([("ws-decoder", None)])
    n = M.NoneError("n")
    s.exception(n)
    assert s.events == [("exception", n.cause)] and s.closing is None
    s = StreamSession([("ws-decoder", None)])
    d = M.DefaultError("d")
    s.exception(d)
    assert s.events == [("exception", d.cause), ("quickClose",)]
    s = StreamSession([("ws-decoder", None)])
    p = M.PlainError("p")
    s.exception(p)
    assert s.events == [("exception", p), ("quickClose",)]
    assert M.NoneError.KIND == CloseType.NONE


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_frame_decoder_host_logic_matches_reference(oracle, seed):
    plan = M.make_plan(seed, 48)
    want = M.run_reference(oracle, plan)
    loop = SelectorLoop()
    ob = M.OracleBatcher(oracle, loop, len(plan))
    got = M.run_dropin(plan, ob, seed=seed)
    for i, (w, g) in enumerate(zip(want, got)):
        assert g == w, (i, plan[i]["dec"], plan[i]["hnd"], w[-4:], g[-4:])
    # the plans exercise every ending
    assert M.endings(want) >= {"GENTLE", "NONE", "DEFAULT", "PLAIN", "InvalidFrameException", "length", "close",
                               "quickClose"}, M.endings(want)
    assert ob.drained_reads > 0  # available() delivered reads still in the batch before it threw
