"""Build the HIP libraries (gfx950) in-tree:
  snf4j_amd/libwsgpu.so      the codec (include/wsgpu.h)
  benchsupport/libwsbench.so synthetic batches + copy ceiling for bench/tests (include/wsbench.h)"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libwsgpu.so")
SOURCES = ["decode.hip", "encode.hip", "aggregate.hip", "api.hip", "batcher.hip", "inflate.hip", "handshake.hip"]
HEADERS = ["ws_rules.h", "wsgpu_internal.h", "wsgpu_scan.h", "../../include/wsgpu.h"]
BENCH_DIR = os.path.join(os.path.dirname(HERE), "benchsupport")
BENCH_SRC = os.path.join(BENCH_DIR, "csrc", "synth.hip")
BENCH_OUT = os.path.join(BENCH_DIR, "libwsbench.so")
BENCH_HDR = os.path.join(os.path.dirname(HERE), "include", "wsbench.h")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -disable-promote-alloca-to-lds: a dynamically indexed local array must not turn
# into an LDS allocation, which slows the dispatch of the piece kernels' millions
# of one-wave workgroups (measured: k_piecesN -10%)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
         "-mllvm", "-disable-promote-alloca-to-lds"]


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps)


def build_bench(force: bool = False) -> str:
    if not force and os.path.exists(BENCH_OUT) and all(
            os.path.getmtime(d) <= os.path.getmtime(BENCH_OUT) for d in (BENCH_SRC, BENCH_HDR)):
        return BENCH_OUT
    tmp = BENCH_OUT + ".tmp"
    r = subprocess.run([HIPCC, *FLAGS, "-shared", BENCH_SRC, "-o", tmp], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {BENCH_SRC}:\n{r.stderr}")
    os.replace(tmp, BENCH_OUT)
    return BENCH_OUT


def build(force: bool = False, verbose: bool = False) -> str:
    build_bench(force)
    if not force and not _stale():
        return OUT
    objdir = os.path.join(HERE, "_build")
    os.makedirs(objdir, exist_ok=True)

    def cc(src):
        obj = os.path.join(objdir, src.replace(".hip", ".o"))
        cmd = [HIPCC, *FLAGS, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        return obj

    with ThreadPoolExecutor(max_workers=4) as ex:
        objs = list(ex.map(cc, SOURCES))
    tmp = OUT + ".tmp"
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
