#!/usr/bin/env python3
"""Linker version script exporting exactly the functions the given C headers
declare (and nothing else: every C++ internal stays local).

  libvortex_amd.so         vx_hash.h                          (the drop-in ABI)
  libvortex_amd_tuning.so  vx_hash.h + vx_tuning.h + vx_synth.h (tests, bench)

tests/test_abi.py checks the built libraries' dynamic symbols against the
same parse of the headers."""
import re
import sys

DECL = re.compile(r"^[A-Za-z_][\w ]*?[\s*]+(vx_\w+)\s*\(", re.M)


def declared(path: str) -> list:
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)  # comments may quote calls
    return sorted(set(DECL.findall(text)))


if __name__ == "__main__":
    names = sorted({n for h in sys.argv[1:] for n in declared(h)})
    print("{\n  global:\n" + "".join(f"    {n};\n" for n in names) + "  local: *;\n};")
