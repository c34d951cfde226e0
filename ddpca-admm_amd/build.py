"""In-tree build of libddpca_amd.so (hipcc, gfx950) -- no JIT cache, no pip install.

Every translation unit under csrc/ is compiled by hipcc (``--offload-arch=gfx950`` for the
.hip device sources) into build/obj and linked into ``libddpca_amd.so`` next to this file, so
the built library travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import threading
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
OBJ = HERE / "build" / "obj"
# experiment builds (A/B of a kernel change): DDPCA_BUILD_DEFINES="-DFOO=1" DDPCA_BUILD_OUT=libx.so
# produce a second library next to this file; load it with DDPCA_AMD_LIB=<path>
LIB = HERE / os.environ.get("DDPCA_BUILD_OUT", "libddpca_amd.so")
PROBE = HERE / "probe"
PROBE_LIB = HERE / "libddpca_probe.so"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = str(ROCM / "bin" / "hipcc")
ARCH = "gfx950"

COMMON = ["-O3", "-std=c++17", "-fPIC", "-fopenmp", "-Wall", "-Wno-unused-function",
          "-Wno-unknown-pragmas", f"-I{HERE.parent / 'include'}", f"-I{CSRC}",
          *os.environ.get("DDPCA_BUILD_DEFINES", "").split()]
DEVICE = [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
LINK = ["-shared", "-fopenmp", f"--offload-arch={ARCH}", f"-L{ROCM / 'lib'}", "-lamdhip64", "-lrccl", "-lrocsolver", "-lrocblas",
        f"-Wl,-rpath,{ROCM / 'lib'}", f"-Wl,-rpath,{ROCM / 'llvm' / 'lib'}"]


def _sources() -> list[Path]:
    return sorted(list(CSRC.glob("*.cpp")) + list(CSRC.glob("*.hip")))


def _digest(src: Path, flags: list[str]) -> str:
    h = hashlib.sha1(" ".join(flags).encode())
    h.update(src.read_bytes())
    for hdr in sorted(CSRC.glob("*.hpp")) + sorted((HERE.parent / "include").glob("*.h")):
        h.update(hdr.read_bytes())
    return h.hexdigest()[:16]


def _compile(src: Path) -> Path:
    flags = COMMON + (DEVICE if src.suffix == ".hip" else [])
    if src.suffix == ".hip":
        flags = flags + ["-x", "hip"]
    obj = OBJ / f"{src.stem}.{_digest(src, flags)}.o"
    if not obj.exists():
        # compile to a private name and rename on success: a killed compile never leaves a
        # truncated object under the cache name, and concurrent builds do not share a file
        tmp = obj.with_suffix(f".{os.getpid()}.{threading.get_ident()}.tmp")
        cmd = [HIPCC, *flags, "-c", str(src), "-o", str(tmp)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            tmp.unlink(missing_ok=True)
            raise RuntimeError(f"compile failed: {src.name}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, obj)
    return obj


def _link(objs: list[Path], out: Path, link: list[str], verbose: bool) -> Path:
    stamp = hashlib.sha1("".join(o.name for o in objs).encode()).hexdigest()[:16]
    stamp_file = OBJ / f"link.{out.name}.stamp"
    if out.exists() and stamp_file.exists() and stamp_file.read_text() == stamp:
        return out
    tmp = out.with_suffix(f".so.{os.getpid()}.tmp")
    cmd = [HIPCC, *[str(o) for o in objs], *link, "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    stamp_file.write_text(stamp)
    if verbose:
        print(f"built {out}", file=sys.stderr)
    return out


def build(verbose: bool = False) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    srcs = _sources()
    probe = sorted(PROBE.glob("*.hip"))
    jobs = min(len(srcs) + len(probe), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(_compile, srcs + probe))
    _link(objs[:len(srcs)], LIB, LINK, verbose)
    # the measurement probes (STREAM ceiling, grid barrier): a library of their own beside the
    # product, linked against it for the error plumbing
    if LIB.name == "libddpca_amd.so":
        _link(objs[len(srcs):], PROBE_LIB, LINK + [f"-L{HERE}", "-lddpca_amd", "-Wl,-rpath,$ORIGIN"], verbose)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
