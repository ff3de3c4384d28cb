"""Build the in-tree HIP library (gfx950) and the oracle checker libraries."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def build_codec(jobs: int = 8) -> str:
    subprocess.run(["make", "-s", "-j", str(jobs), "-C", os.path.join(HERE, "csrc")], check=True)
    return os.path.join(HERE, "libstg_codec.so")


def build_oracle(ref: bool | None = None) -> None:
    import sys
    sys.path.insert(0, ROOT)
    from oracle.oracle import build
    build(ref=ref)


if __name__ == "__main__":
    print(build_codec())
    build_oracle()
