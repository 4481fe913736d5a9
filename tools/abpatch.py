#!/usr/bin/env python3
"""Build a measurement variant of libnbgpu.so from a patched copy of the working tree's sources.

  python tools/abpatch.py NAME FILE 'old text' 'new text' [FILE 'old' 'new' ...]

Copies netbricks_amd/csrc + include into tools/ab/src_NAME, applies each exact, unique text
replacement to FILE (a path under netbricks_amd/csrc), and builds tools/ab/lib_NAME.so.  Ablations
(timing only: the results of such a build are wrong by design) and A/B variants live only there; the
product source is never modified.  Load a variant with NBG_LIB_OVERRIDE=tools/ab/lib_NAME.so.
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    if len(sys.argv) < 5 or (len(sys.argv) - 2) % 3:
        raise SystemExit(__doc__)
    name = sys.argv[1]
    src = os.path.join(ROOT, "tools", "ab", f"src_{name}")
    lib = os.path.join(ROOT, "tools", "ab", f"lib_{name}.so")
    if os.path.isdir(src):
        shutil.rmtree(src)
    os.makedirs(os.path.join(src, "netbricks_amd"))
    shutil.copytree(os.path.join(ROOT, "netbricks_amd", "csrc"), os.path.join(src, "netbricks_amd", "csrc"),
                    ignore=shutil.ignore_patterns("*.o", "*.s"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(src, "include"))
    args = sys.argv[2:]
    for i in range(0, len(args), 3):
        f = os.path.join(src, "netbricks_amd", "csrc", args[i])
        old, new = args[i + 1].encode().decode("unicode_escape"), args[i + 2].encode().decode("unicode_escape")
        with open(f) as fh:
            s = fh.read()
        if s.count(old) != 1:
            raise SystemExit(f"abpatch: {args[i]}: the text occurs {s.count(old)} times: {old[:80]!r}")
        with open(f, "w") as fh:
            fh.write(s.replace(old, new))
    subprocess.check_call(["make", "-s", "-C", os.path.join(src, "netbricks_amd", "csrc"), f"OUT={lib}"])
    print("built", lib)


if __name__ == "__main__":
    main()
