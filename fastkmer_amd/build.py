"""Build the HIP library and CLI in-tree for gfx950 (no JIT cache).

  fastkmer_amd/lib/libfastkmer.so   C-ABI (include/fastkmer.h)
  fastkmer_amd/bin/fastkmer-cli     LocalTestKmerCounter-compatible driver

Usage: python -m fastkmer_amd.build [--force]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib", "libfastkmer.so")
CLI = os.path.join(PKG, "bin", "fastkmer-cli")
ARCH = os.environ.get("FASTKMER_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

LIB_SOURCES = ["fk_kernels.hip", "fk_api.cpp", "fk_comm.cpp", "fk_split.cpp"]
DEPS = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".inc", ".h")) or f in ("fk_api.cpp", "fk_comm.cpp", "fk_split.cpp"))


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


RESOURCES = os.path.join(PKG, "lib", "kernel_resources.txt")


def _resource_table(remarks: str) -> list[dict]:
    """Per-kernel registers / scratch / occupancy / LDS from clang's
    -Rpass-analysis=kernel-resource-usage remarks."""
    import re
    rows, cur = [], None
    for line in remarks.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"kernel": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"LDS Size \[bytes/block\]|VGPRs Spill|SGPRs Spill): (\d+)", line)
        if m and cur is not None:
            name = m.group(1)
            cur[name if "Spill" in name else name.split(" ")[0]] = int(m.group(2))
    return rows


def _compile_kernels(src: str, obj: str, defs: list[str] = ()) -> None:
    """Compile the kernel file with resource-usage remarks; no kernel may use
    scratch (a spilled register array costs a global-memory round trip per
    access, e.g. 1.57 -> 2.38 ms for the signature kernel)."""
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall",
           "-Wno-unused-function", *defs, "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", obj]
    print("+", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, stderr=subprocess.PIPE, text=True)
    rows = _resource_table(r.stderr)
    other = "\n".join(l for l in r.stderr.splitlines() if "kernel-resource-usage" not in l and l.strip()
                      and not l.lstrip().startswith(("|", "^")) and not re.match(r"\s*\d+ \|", l))
    if other:
        print(other, file=sys.stderr)
    if r.returncode != 0:
        raise subprocess.CalledProcessError(r.returncode, cmd)
    resources = os.path.join(os.path.dirname(obj), "kernel_resources.txt")
    with open(resources, "w") as f:
        f.write("kernel\tVGPRs\tAGPRs\tscratch_B_per_lane\toccupancy_waves_per_SIMD\tLDS_B\n")
        for row in rows:
            f.write("\t".join(str(row.get(c, "")) for c in
                               ("kernel", "VGPRs", "AGPRs", "ScratchSize", "Occupancy", "LDS")) + "\n")
    bad = [row["kernel"] for row in rows if row.get("ScratchSize", 0) or row.get("VGPRs Spill", 0)]
    if bad:
        raise RuntimeError(f"kernels using scratch memory (see {resources}): {bad}")


PROBES_LIB = os.path.join(PKG, "lib_probes", "libfastkmer.so")


def _build_lib(lib: str, deps: list[str], force: bool, defs: list[str]) -> None:
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    if not (force or _stale(lib, deps)):
        return
    objs = []
    for src in LIB_SOURCES:
        obj = os.path.join(os.path.dirname(lib), os.path.splitext(src)[0] + ".o")
        if src.endswith(".hip"):
            _compile_kernels(os.path.join(CSRC, src), obj, defs)
        else:
            _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
                  "-Wall", "-Wno-unused-function", *defs, "-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj])
        objs.append(obj)
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs, "-ldl"])
    for o in objs:
        os.remove(o)


def build_probes(force: bool = False) -> str:
    """A measurement-only library with the result-altering timing probes compiled in (-DFK_PROBES:
    FASTKMER_FUSED_PROBE, FASTKMER_DEBUG_PHASE, FASTKMER_SPLIT_MAP, the host trace
    FASTKMER_HOST_TRACE and the map phase stamps).
    Scripts select it with FASTKMER_LIB; nothing else loads it."""
    deps = [os.path.join(CSRC, d) for d in DEPS] + [os.path.join(ROOT, "include", "fastkmer.h")]
    _build_lib(PROBES_LIB, deps, force, ["-DFK_PROBES"])
    return PROBES_LIB


def build(force: bool = False) -> str:
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    os.makedirs(os.path.dirname(CLI), exist_ok=True)
    deps = [os.path.join(CSRC, d) for d in DEPS] + [os.path.join(ROOT, "include", "fastkmer.h")]
    _build_lib(LIB, deps, force, [])
    if force or _stale(CLI, [os.path.join(CSRC, "fk_cli.cpp"), LIB]):
        _run(["g++", "-O2", "-std=c++17", "-o", CLI, os.path.join(CSRC, "fk_cli.cpp"),
              f"-L{os.path.dirname(LIB)}", "-lfastkmer", "-Wl,-rpath,$ORIGIN/../lib"])
    build_jni(force)
    return LIB


JNI_SRC = os.path.join(ROOT, "jni", "fastkmer_jni.c")
JNI_LIB = os.path.join(PKG, "lib", "libfastkmer_jni.so")


def jni_include_dirs() -> list[str]:
    """JDK include directories ($JAVA_HOME or a JDK under /usr/lib/jvm), [] when no jni.h exists."""
    homes = [os.environ.get("JAVA_HOME", "")]
    if os.path.isdir("/usr/lib/jvm"):
        homes += [os.path.join("/usr/lib/jvm", d) for d in sorted(os.listdir("/usr/lib/jvm"))]
    for h in homes:
        inc = os.path.join(h, "include") if h else ""
        if inc and os.path.exists(os.path.join(inc, "jni.h")):
            return [inc, os.path.join(inc, "linux")]
    return []


def build_jni(force: bool = False) -> str | None:
    """The JNI shim (jni/fastkmer_jni.c) for skc.gpu.NativeKmerCounter, only where a JDK is
    installed (this image has none: the shim is then not built)."""
    incs = jni_include_dirs()
    if not incs:
        return None
    if force or _stale(JNI_LIB, [JNI_SRC, LIB, os.path.join(ROOT, "include", "fastkmer.h")]):
        _run(["gcc", "-O2", "-shared", "-fPIC", *[f"-I{d}" for d in incs], f"-I{os.path.join(ROOT, 'include')}",
              JNI_SRC, f"-L{os.path.dirname(LIB)}", "-lfastkmer", "-Wl,-rpath,$ORIGIN", "-o", JNI_LIB])
    return JNI_LIB


def build_variant(name: str, defs: list[str], force: bool = False) -> str:
    """An A/B build of the library with extra -D flags into fastkmer_amd/lib_<name>/ (measurement
    only: scripts select it with FASTKMER_LIB)."""
    lib = os.path.join(PKG, f"lib_{name}", "libfastkmer.so")
    deps = [os.path.join(CSRC, d) for d in DEPS] + [os.path.join(ROOT, "include", "fastkmer.h")]
    _build_lib(lib, deps, force, defs)
    return lib


if __name__ == "__main__":
    if "--probes" in sys.argv:
        build_probes(force="--force" in sys.argv)
    elif "--variant" in sys.argv:  # python -m fastkmer_amd.build --variant NAME -DX=1 ...
        i = sys.argv.index("--variant")
        build_variant(sys.argv[i + 1], [a for a in sys.argv[i + 2:] if a.startswith("-D")],
                      force="--force" in sys.argv)
    else:
        build(force="--force" in sys.argv)
