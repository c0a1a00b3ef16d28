"""bench.py's launcher contract (CPU only, nothing touches a GPU): under a launcher,
--gpus must equal WORLD_SIZE, so a line can never report fewer GPUs than asked for."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=120)


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "8"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 8 but WORLD_SIZE=1" in r.stderr


def test_config_choices_and_overrides():
    sys.path.insert(0, ROOT)
    import bench
    argv = sys.argv
    try:
        sys.argv = ["bench.py", "--config", "3"]
        a = bench.parse()
        assert (a.frames, a.payload, a.sessions, a.binary) == (8 << 20, 4096, 1024, False)
        sys.argv = ["bench.py", "--config", "1", "--frames", "4096"]
        a = bench.parse()
        assert (a.frames, a.payload, a.sessions, a.binary) == (4096, 1024, 256, True)
        sys.argv = ["bench.py"]
        a = bench.parse()
        assert (a.frames, a.payload, a.sessions, a.binary, a.gpus) == (1 << 20, 4096, 1024, False, None)
    finally:
        sys.argv = argv


def test_cpu_threads_from_affinity(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    aff = len(os.sched_getaffinity(0))
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    assert bench.cpu_threads()[0] == aff
    if aff > 1:
        monkeypatch.setenv("OMP_NUM_THREADS", "1")
        assert bench.cpu_threads()[0] == 1


def test_bench_inflight_limit_is_the_library_one():
    import bench
    from snf4j_amd import _lib
    assert bench.BATCHER_MAX_INFLIGHT == _lib.BATCHER_MAX_INFLIGHT
