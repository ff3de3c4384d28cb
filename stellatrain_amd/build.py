"""Build the in-tree HIP library (gfx950) and the oracle checker libraries."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def build_codec(jobs: int = 8) -> str:
    subprocess.run(["make", "-s", "-j", str(jobs), "-C", os.path.join(HERE, "csrc")], check=True)
    return os.path.join(HERE, "libstg_codec.so")


def build_concurrency() -> str:
    """tests/cpp/concurrency: T threads on one codec handle through the shim
    (test binary, run by tests/test_gpu_concurrency.py on the GPU box)."""
    exe = os.path.join(ROOT, "tests", "cpp", "concurrency")
    subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "concurrency.cpp"), "-o", exe, "-L", HERE, "-lstg_codec",
                    "-lpthread", "-Wl,-rpath,$ORIGIN/../../stellatrain_amd"], check=True)
    return exe


def build_shim() -> str:
    """tests/cpp/shim_factory: the reference engine's codec factory and MERGE
    call site compiled against include/stg/compressor.h (test binary, run by
    tests/test_gpu_api.py on the GPU box)."""
    exe = os.path.join(ROOT, "tests", "cpp", "shim_factory")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "shim_factory.cpp"), "-o", exe, "-L", HERE, "-lstg_codec",
                    "-Wl,-rpath,$ORIGIN/../../stellatrain_amd"], check=True)
    return exe


def build_oracle(ref: bool | None = None) -> None:
    import sys
    sys.path.insert(0, ROOT)
    from oracle.oracle import build
    build(ref=ref)


if __name__ == "__main__":
    print(build_codec())
    build_oracle()
    print(build_shim())
    print(build_concurrency())
