"""Reproducible build check of libfedagg.so (build container, CPU only).

Builds the library twice from copies of the sources in two different
directories, with __graft_entry__.HIP_FLAGS (which fix the compilation-unit id
instead of hipcc's random one), and compares the md5 of both builds with each
other and with the in-tree library.  bench.py reports the stored PMC traffic
only for a library of the md5 that summary profiled, so an identical rebuild
must keep that md5.

python tools/repro_build.py [--out profiles/r05_repro_build.json]
"""
import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402


def md5(path):
    h = hashlib.md5()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def build_copy(root):
    for sub in ("fedsim_amd/csrc", "include"):
        shutil.copytree(os.path.join(REPO, sub), os.path.join(root, sub))
    out = os.path.join(root, "fedsim_amd", "libfedagg.so")
    src = os.path.join(root, "fedsim_amd", "csrc", "fedagg_kernels.hip")
    t0 = time.time()
    subprocess.check_call([G.HIPCC, *G.HIP_FLAGS, "-o", out, src], cwd=root)
    return md5(out), round(time.time() - t0, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r05_repro_build.json"))
    a = ap.parse_args()
    builds = []
    for name in ("a", "b"):
        with tempfile.TemporaryDirectory(prefix=f"repro_{name}_") as d:
            m, dt = build_copy(d)
            builds.append(dict(dir=d, md5=m, seconds=dt))
    lib = os.path.join(REPO, "fedsim_amd", "libfedagg.so")
    in_tree = md5(lib) if os.path.exists(lib) else None
    rec = dict(flags=G.HIP_FLAGS, builds=builds, in_tree_md5=in_tree,
               identical=builds[0]["md5"] == builds[1]["md5"],
               in_tree_matches=in_tree == builds[0]["md5"])
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))
    sys.exit(0 if rec["identical"] else 1)


if __name__ == "__main__":
    main()
