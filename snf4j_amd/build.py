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
SOURCES = ["decode.hip", "encode.hip", "aggregate.hip", "api.hip", "batcher.hip", "inflate.hip", "handshake.hip", "deflate.hip"]
HEADERS = ["ws_rules.h", "wsgpu_internal.h", "wsgpu_scan.h", "deflate_core.h", "deflate_pmd.h", "../../include/wsgpu.h"]
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


def _digest(paths, flags) -> str:
    """sha256 of the sources, headers and compile flags a library is built from."""
    import hashlib
    h = hashlib.sha256(" ".join(flags).encode())
    for p in paths:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _fresh(out: str, digest: str) -> bool:
    """The library exists and was built from exactly these sources (its .srchash
    sidecar): a binary pushed with other sources is rebuilt, whatever the mtimes."""
    try:
        with open(out + ".srchash") as fh:
            return os.path.exists(out) and fh.read().strip() == digest
    except OSError:
        return False


def _record(out: str, digest: str) -> None:
    with open(out + ".srchash", "w") as fh:
        fh.write(digest + "\n")


def build_bench(force: bool = False) -> str:
    digest = _digest([BENCH_SRC, BENCH_HDR], FLAGS)
    if not force and _fresh(BENCH_OUT, digest):
        return BENCH_OUT
    tmp = BENCH_OUT + ".tmp"
    r = subprocess.run([HIPCC, *FLAGS, "-shared", BENCH_SRC, "-o", tmp], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {BENCH_SRC}:\n{r.stderr}")
    os.replace(tmp, BENCH_OUT)
    _record(BENCH_OUT, digest)
    return BENCH_OUT


def build(force: bool = False, verbose: bool = False) -> str:
    build_bench(force)
    digest = _digest([os.path.join(CSRC, s) for s in SOURCES + HEADERS], FLAGS)
    if not force and _fresh(OUT, digest):
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
    _record(OUT, digest)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
