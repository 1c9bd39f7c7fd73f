#!/usr/bin/env python3
"""Build the product library of another git revision as an A/B variant
(lib/variants/<name>.so), from that revision's csrc/ and include/ (git archive into /tmp).

usage: python tools/build_rev.py <rev> <name> [-DX=1 ...]
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "access-control-srv_amd")]
from acs_mi355x import build  # noqa: E402


def main():
    rev, name, defines = sys.argv[1], sys.argv[2], sys.argv[3:]
    tmp = tempfile.mkdtemp(prefix="acs_rev_")
    arc = subprocess.run(["git", "-C", ROOT, "archive", rev, "access-control-srv_amd/csrc", "include"],
                         check=True, capture_output=True).stdout
    subprocess.run(["tar", "-x", "-C", tmp], input=arc, check=True)
    csrc = os.path.join(tmp, "access-control-srv_amd", "csrc")
    build.CSRC, build.ROOT = csrc, tmp  # _hipcc's include paths
    out = os.path.join(build.PKG, "lib", "variants", name + ".so")
    hosts = [os.path.join(csrc, os.path.basename(h)) for h in build._HOST_SRCS]
    build._hipcc(os.path.join(csrc, "acs_kernels.hip"), out, tuple(defines), host_srcs=hosts)
    print(out)


if __name__ == "__main__":
    main()
