"""In-tree native build of ``video_edge_ai_proxy_amd._vep`` for gfx950.

Every source (host C++ and HIP) is compiled with ``hipcc --offload-arch=gfx950``; the module is
linked in-tree so it travels with the repo snapshot to the GPU box. Incremental: an object is
rebuilt when its source or any header under csrc/ is newer.

    python csrc/build.py [--clean] [-j N] [--debug]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
PKG = ROOT / "video_edge_ai_proxy_amd"
OBJ = ROOT / "build" / "obj"
ARCH = os.environ.get("VEP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def module_path() -> Path:
    return PKG / f"_vep{ext_suffix()}"


def sources() -> list[Path]:
    out = sorted(CSRC.glob("*.cpp")) + sorted((CSRC / "vep").glob("*.cpp"))
    out += sorted((CSRC / "vep").glob("*.hip"))
    return out


def _flags(debug: bool) -> list[str]:
    import pybind11

    inc = [
        f"-I{CSRC}",
        f"-I{pybind11.get_include()}",
        f"-I{sysconfig.get_paths()['include']}",
    ]
    opt = ["-O1", "-g"] if debug else ["-O3", "-gline-tables-only", "-Xarch_host", "-march=x86-64-v3"]  # line tables: hostprof; v3: BMI2/LZCNT in the CABAC renorm (any EPYC)
    return [
        f"--offload-arch={ARCH}",
        "-std=c++17",
        "-fPIC",
        "-fvisibility=hidden",
        "-Wall",
        "-Wno-unused-result",
        "-Wno-unused-function",
        *opt,
        *inc,
    ]


def _newest_header() -> float:
    hs = list(CSRC.rglob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, obj: Path, flags: list[str]) -> tuple[Path, str]:
    cmd = [HIPCC, *flags, "-c", str(src), "-o", str(obj)]
    if src.suffix == ".hip":
        cmd[1:1] = ["-x", "hip"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj, r.stderr


def build(jobs: int | None = None, debug: bool = False, verbose: bool = False) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    flags = _flags(debug)
    hdr = _newest_header()
    todo = []
    objs = []
    for s in sources():
        o = OBJ / (s.relative_to(CSRC).as_posix().replace("/", "__") + ".o")
        objs.append(o)
        if not o.exists() or o.stat().st_mtime < max(s.stat().st_mtime, hdr):
            todo.append((s, o))
    jobs = jobs or min(8, os.cpu_count() or 4)
    if todo:
        with cf.ThreadPoolExecutor(jobs) as ex:
            futs = [ex.submit(_compile, s, o, flags) for s, o in todo]
            for f in cf.as_completed(futs):
                o, err = f.result()
                if verbose and err.strip():
                    print(err, file=sys.stderr)
    out = module_path()
    if todo or not out.exists() or out.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        tmp = out.with_suffix(".tmp.so")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp),
               "-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, out)
    return out


STUB_SRC = CSRC / "tests" / "rocdec_stub.cpp"
STUB = ROOT / "tests" / "native" / "libvep_rocdec_stub.so"


def build_rocdec_stub() -> Path:
    """Test double of librocdecode (csrc/tests/rocdec_stub.cpp) for the VCN backend tests, linked
    against the data-plane objects of build(); kept in-tree so GPU boxes receive it."""
    flags = _flags(False)
    obj = OBJ / "tests__rocdec_stub.cpp.o"
    vep_objs = [OBJ / (s.relative_to(CSRC).as_posix().replace("/", "__") + ".o")
                for s in sources() if s.parent.name == "vep"]
    if not obj.exists() or obj.stat().st_mtime < max(STUB_SRC.stat().st_mtime, _newest_header()):
        _compile(STUB_SRC, obj, flags)
    newest = max(o.stat().st_mtime for o in [obj, *vep_objs])
    if not STUB.exists() or STUB.stat().st_mtime < newest:
        STUB.parent.mkdir(parents=True, exist_ok=True)
        tmp = STUB.with_suffix(".tmp.so")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", str(obj), *map(str, vep_objs), "-o", str(tmp),
               "-lpthread", "-Wl,--no-undefined"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"stub link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, STUB)
    return STUB


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    if a.clean:
        shutil.rmtree(OBJ, ignore_errors=True)
        module_path().unlink(missing_ok=True)
    p = build(a.j, a.debug, a.v)
    print(p)
    print(build_rocdec_stub())


if __name__ == "__main__":
    main()
