"""Build libdlsa_hip.so in-tree for gfx950 (MI355X).

    python -m dlsa_amd.build [--force] [--verbose]

hipcc cross-compiles without a GPU, so this runs in the build container; the
resulting .so travels to the GPU box with the repository snapshot.
"""

from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libdlsa_hip.so")
SOURCES = (["irls_coop.hip"] + [f"irls_coop_g{i}.hip" for i in range(1, 7)] +
           ["irls_wave.hip", "irls_wave_g2.hip", "irls_oz.hip", "irls_oz_g2.hip"] +
           ["wide_pass.hip", "wide_oz.hip", "cat_pass.hip", "partition_rows.hip", "moments.hip", "ols_stream.hip", "eval_pass.hip", "newton_solve.hip", "aux_kernels.hip", "capi.hip", "lars_host.cpp"])
HEADERS = ["dlsa_internal.hpp", "irls_coop_impl.hpp", "irls_wave_impl.hpp", "irls_oz_impl.hpp", os.path.join("..", "..", "include", "dlsa_hip.h")]
ARCH = os.environ.get("DLSA_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm >= 7 required)")


def _common_flags() -> list:
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
            "-Wno-unused-function", "-Wno-unused-command-line-argument",
            "-I" + os.path.join(ROOT, "include")]


def _toolchain_key() -> str:
    """Target architecture + a hash of the compile flags and the resolved
    compiler / ROCm install: objects and the library built under another key
    are not reused."""
    import hashlib
    h = hashlib.sha1("\0".join(_common_flags() + [os.path.realpath(hipcc()),
                                                  os.path.realpath("/opt/rocm")]).encode())
    return f"{ARCH}-{h.hexdigest()[:12]}"


BUILD_DIR = os.path.join(ROOT, "build")
STAMP = os.path.join(BUILD_DIR, "libdlsa_hip.key")  # toolchain key of the in-tree .so


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    try:
        with open(STAMP) as f:
            if f.read().strip() != _toolchain_key():
                return True
    except OSError:
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps)


def _obj_cache() -> str:
    return os.path.join(BUILD_DIR, "obj", _toolchain_key())


def _cached_object(src: str) -> str | None:
    """The object of `src` from the last product build (no defines) under the
    current toolchain key, if it is newer than the source and every header."""
    obj = os.path.join(_obj_cache(), os.path.splitext(src)[0] + ".o")
    if not os.path.exists(obj):
        return None
    t = os.path.getmtime(obj)
    deps = [os.path.join(CSRC, src)] + [os.path.join(CSRC, h) for h in HEADERS] + [__file__]
    return obj if all(os.path.getmtime(d) <= t for d in deps) else None


def build(force: bool = False, verbose: bool = False, out: str = OUT, defines=(),
          only=None) -> str:
    """Compile every source to an object in parallel, then link the .so.

    Profiling variants (out != OUT) may name `only`: the sources the defines
    apply to; the other objects are taken from the product build's object
    cache (build/obj) when it is current."""
    if not force and out == OUT and not _stale():
        return OUT
    import tempfile
    from concurrent.futures import ThreadPoolExecutor

    common = [hipcc()] + _common_flags()
    product = out == OUT and not defines
    jobs = int(os.environ.get("DLSA_BUILD_JOBS", min(8, os.cpu_count() or 1)))
    with tempfile.TemporaryDirectory(prefix="dlsa_build_") as tmp:
        def compile_one(src):
            # reuse the cached object of a source whose object is current: the
            # variant builds' untouched sources, and an incremental product build
            if (only is not None and src not in only) or (product and not force):
                cached = _cached_object(src)
                if cached:
                    return cached, None
            obj = os.path.join(tmp, os.path.splitext(src)[0] + ".o")
            cmd = common + ([f"-D{d}" for d in defines] if only is None or src in only else [])
            cmd = cmd + ["-c", os.path.join(CSRC, src), "-o", obj]
            if src.endswith(".cpp"):  # host-only code (LARS): AVX2/FMA vector loops (x86-64-v3)
                cmd += ["-march=x86-64-v3"]
            if verbose:
                print(" ".join(cmd), flush=True)
            return obj, subprocess.run(cmd, capture_output=True, text=True)

        with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            results = list(ex.map(compile_one, SOURCES))
        for obj, res in results:
            if res is not None and res.returncode != 0:
                sys.stderr.write(res.stdout + res.stderr)
                raise RuntimeError(f"hipcc failed on {obj} ({res.returncode})")
        if product:  # keep the objects for variant builds
            cache = _obj_cache()
            os.makedirs(cache, exist_ok=True)
            for obj, res in results:
                if res is not None:
                    shutil.copy2(obj, os.path.join(cache, os.path.basename(obj)))
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC",
               *[o for o, _ in results], "-o", out + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            sys.stderr.write(res.stdout + res.stderr)
            raise RuntimeError(f"link failed ({res.returncode})")
    # every symbol must resolve at load time: a kernel template whose host
    # stub the compiler silently dropped links fine and only fails at dlopen
    # (checked in a child process, so this one keeps no HIP library loaded)
    chk = subprocess.run([sys.executable, "-c",
                          "import ctypes, os, sys; ctypes.CDLL(sys.argv[1], mode=os.RTLD_NOW)",
                          out + ".tmp"], capture_output=True, text=True)
    if chk.returncode != 0:
        sys.stderr.write(chk.stderr)
        raise RuntimeError(f"{out}.tmp does not load (unresolved symbols)")
    os.replace(out + ".tmp", out)
    if out == OUT and not defines:
        os.makedirs(BUILD_DIR, exist_ok=True)
        with open(STAMP, "w") as f:
            f.write(_toolchain_key() + "\n")
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)
    print(build(force=a.force, verbose=a.verbose))


if __name__ == "__main__":
    main()
