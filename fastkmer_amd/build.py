"""Build the HIP library and CLI in-tree for gfx950 (no JIT cache).

  fastkmer_amd/lib/libfastkmer.so   C-ABI (include/fastkmer.h)
  fastkmer_amd/bin/fastkmer-cli     LocalTestKmerCounter-compatible driver

Usage: python -m fastkmer_amd.build [--force]
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib", "libfastkmer.so")
CLI = os.path.join(PKG, "bin", "fastkmer-cli")
ARCH = os.environ.get("FASTKMER_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

LIB_SOURCES = ["fk_kernels.hip", "fk_api.cpp"]
DEPS = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".inc", ".h")) or f == "fk_api.cpp")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build(force: bool = False) -> str:
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    os.makedirs(os.path.dirname(CLI), exist_ok=True)
    deps = [os.path.join(CSRC, d) for d in DEPS] + [os.path.join(ROOT, "include", "fastkmer.h")]
    if force or _stale(LIB, deps):
        objs = []
        for src in LIB_SOURCES:
            obj = os.path.join(PKG, "lib", os.path.splitext(src)[0] + ".o")
            lang = ["-x", "hip"] if src.endswith(".cpp") else []
            _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
                  "-Wall", "-Wno-unused-function", *lang, "-c", os.path.join(CSRC, src), "-o", obj])
            objs.append(obj)
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs])
        for o in objs:
            os.remove(o)
    if force or _stale(CLI, [os.path.join(CSRC, "fk_cli.cpp"), LIB]):
        _run(["g++", "-O2", "-std=c++17", "-o", CLI, os.path.join(CSRC, "fk_cli.cpp"),
              f"-L{os.path.dirname(LIB)}", "-lfastkmer", "-Wl,-rpath,$ORIGIN/../lib"])
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
