"""The ctypes mirrors of the C-ABI structs (dlsa_amd/_hip.py) against the
header itself: a C probe compiled with gcc from include/dlsa_hip.h prints
sizeof / offsetof of every field; the ctypes layout must match, so a field
added on one side only fails here instead of shifting the stats read back."""

import shutil
import subprocess

import pytest

from dlsa_amd import _hip

INCLUDE = __import__("pathlib").Path(__file__).resolve().parents[1] / "include"


def _probe(tmp_path, struct, fields):
    src = tmp_path / "probe.c"
    lines = ["#include <stddef.h>", "#include <stdio.h>", '#include "dlsa_hip.h"',
             "int main(void) {", f'  printf("size %zu\\n", sizeof({struct}));']
    for f in fields:
        lines.append(f'  printf("{f} %zu\\n", offsetof({struct}, {f}));')
    lines += ["  return 0;", "}"]
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", str(INCLUDE), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return {k: int(v) for k, v in (line.split() for line in out.splitlines())}


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
@pytest.mark.parametrize("cls,struct", [(_hip.FitStats, "dlsa_fit_stats"),
                                        (_hip.FitOptions, "dlsa_fit_options")])
def test_ctypes_struct_matches_header(tmp_path, cls, struct):
    names = [f for f, _ in cls._fields_]
    c = _probe(tmp_path, struct, names)
    assert c["size"] == __import__("ctypes").sizeof(cls)
    for f in names:
        assert c[f] == getattr(cls, f).offset, f
