"""Native build driver for the grace_amd HIP/C++ extension (``grace_amd/_C.so``).

No setuptools/cpp_extension indirection and no source translation: every ``.hip`` and
``.cpp`` file under ``csrc/`` is compiled directly by ``hipcc --offload-arch=gfx950`` and
linked against the *torch-bundled* HIP runtime and RCCL (``torch/lib``), so that exactly one
``libamdhip64.so.7`` / ``librccl.so.1`` lives in the process next to PyTorch.

Incremental: an object is rebuilt when its source, any header under ``csrc/include`` or
this file is newer than it.  Objects compile in parallel (``MAX_JOBS``, default 8).

Usage::

    python -m grace_amd._build            # build (incremental)
    python -m grace_amd._build --clean    # rebuild everything
    python -m grace_amd._build --asan     # host-side AddressSanitizer preset -> build/asan/_C.so

The ASan preset instruments the HOST code only (bindings, argument validation, the RCCL runtime
in csrc/comm): every ``-fsanitize=`` sits directly after ``-Xarch_host`` (GPU code objects are
never sanitized -- GPU ASan / xnack+ is not available on the MI355X pool).  Run host-side checks
with tools/asan_host_check.sh (preloads clang's ASan runtime, loads the instrumented library
through ``GRACE_AMD_NATIVE_SO``).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
OUT = ROOT / "grace_amd" / "_C.so"
BUILD_ASAN = ROOT / "build" / "asan_obj"
OUT_ASAN = ROOT / "build" / "asan" / "_C.so"
ASAN_COMPILE = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer", "-g"]
ASAN_LINK = ["-Xarch_host", "-fsanitize=address", "-shared-libasan"]
ARCH = os.environ.get("GRACE_OFFLOAD_ARCH", "gfx950")


def _torch_paths():
    import torch  # noqa: WPS433  (only needed at build time)

    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return tdir / "lib", inc, abi


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (expected /opt/rocm/bin/hipcc)")


def _sources():
    srcs = sorted(CSRC.rglob("*.hip")) + sorted(CSRC.rglob("*.cpp"))
    return [s for s in srcs if "/_disabled/" not in str(s)]


def _common_flags(inc_dirs, abi):
    py_inc = sysconfig.get_paths()["include"]
    flags = [
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-munsafe-fp-atomics",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-DUSE_ROCM=1",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
        "-Wno-unused-command-line-argument",
        f"-I{CSRC / 'include'}",
        "-I/opt/rocm/include",
        f"-I{py_inc}",
    ]
    for d in inc_dirs:
        flags.append(f"-isystem{d}")
    return flags


def _needs_rebuild(src: Path, obj: Path, dep_mtime: float) -> bool:
    if not obj.exists():
        return True
    om = obj.stat().st_mtime
    return src.stat().st_mtime > om or dep_mtime > om


def _compile(hipcc, flags, src: Path, obj: Path):
    obj.parent.mkdir(parents=True, exist_ok=True)
    cmd = [hipcc, *flags, "-c", str(src), "-o", str(obj)]
    if src.suffix == ".cpp":
        cmd[1:1] = ["-x", "hip"]
    t0 = time.time()
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{proc.stdout}\n{proc.stderr}")
    return src.name, time.time() - t0


def build(clean: bool = False, verbose: bool = True, asan: bool = False) -> Path:
    tlib, tinc, abi = _torch_paths()
    hipcc = _hipcc()
    build_dir, out = (BUILD_ASAN, OUT_ASAN) if asan else (BUILD, OUT)
    if clean and build_dir.exists():
        shutil.rmtree(build_dir)
    build_dir.mkdir(parents=True, exist_ok=True)
    out.parent.mkdir(parents=True, exist_ok=True)
    flags = _common_flags(tinc, abi)
    if asan:
        flags = [f for f in flags if f != "-O3"] + ["-O1", *ASAN_COMPILE]
    headers = list((CSRC / "include").rglob("*.h"))
    dep_mtime = max([h.stat().st_mtime for h in headers] + [Path(__file__).stat().st_mtime])
    srcs = _sources()
    objs, todo = [], []
    for s in srcs:
        o = build_dir / (s.relative_to(CSRC).as_posix().replace("/", "__") + ".o")
        objs.append(o)
        if _needs_rebuild(s, o, dep_mtime):
            todo.append((s, o))
    jobs = max(1, int(os.environ.get("MAX_JOBS", "8")))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=min(jobs, len(todo))) as ex:
            futs = [ex.submit(_compile, hipcc, flags, s, o) for s, o in todo]
            for f in cf.as_completed(futs):
                name, dt = f.result()
                if verbose:
                    print(f"[grace_amd build] {name}: {dt:.1f}s", flush=True)
    newest_obj = max(o.stat().st_mtime for o in objs)
    if todo or not out.exists() or out.stat().st_mtime < newest_obj:
        link = [
            hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *(ASAN_LINK if asan else []), "-o", str(out),
            *map(str, objs),
            f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            "-ltorch_python", "-lamdhip64", "-lrccl", f"-Wl,-rpath,{tlib}",
        ]
        proc = subprocess.run(link, capture_output=True, text=True)
        if proc.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(link)}\n{proc.stdout}\n{proc.stderr}")
        if verbose:
            print(f"[grace_amd build] linked {out.relative_to(ROOT)}", flush=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--asan", action="store_true", help="host-side AddressSanitizer build (build/asan/_C.so)")
    args = ap.parse_args(argv)
    build(clean=args.clean, asan=args.asan)


if __name__ == "__main__":
    sys.exit(main())
