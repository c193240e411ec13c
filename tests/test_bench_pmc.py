"""bench.py's roofline.traffic provenance: the committed PMC summary is
reported only for the build of libfedagg.so it was measured on."""
import json

import bench


def _summary(tmp_path, lib_md5):
    d = dict(kernel="k_reduce_narrow<U=8, VW=2>", K=1000, P=25000000, layout="blocked4096",
             step="fused", hbm_bytes_per_launch=100299732991.98772,
             source=dict(lib_md5=lib_md5, profile="profiles/rXX/", host="box"))
    p = tmp_path / "pmc_traffic.json"
    p.write_text(json.dumps(d))
    return str(p)


def _lib(tmp_path, data=b"build A"):
    p = tmp_path / "libfedagg.so"
    p.write_bytes(data)
    return str(p)


ARGS = (1000, 25000000, "k_reduce_narrow<U=8, VW=2>", "blocked4096", "fused")


def test_same_build_reports_traffic(tmp_path):
    lib = _lib(tmp_path)
    t, src = bench.load_pmc(_summary(tmp_path, bench._md5(lib)), *ARGS, lib)
    assert t == 100299732991.98772
    assert src["lib_md5"] == src["lib_md5_loaded"] and src["profile"] == "profiles/rXX/"


def test_other_build_reports_null(tmp_path):
    lib = _lib(tmp_path)
    t, src = bench.load_pmc(_summary(tmp_path, "0" * 32), *ARGS, lib)
    assert t is None and "another build" in src["reason"]


def test_summary_without_build_id_reports_null(tmp_path):
    lib = _lib(tmp_path)
    t, src = bench.load_pmc(_summary(tmp_path, None), *ARGS, lib)
    assert t is None


def test_other_workload_reports_null(tmp_path):
    lib = _lib(tmp_path)
    t, src = bench.load_pmc(_summary(tmp_path, bench._md5(lib)), 500, *ARGS[1:], lib)
    assert t is None and "workload" in src["reason"]


def test_missing_summary(tmp_path):
    t, src = bench.load_pmc(str(tmp_path / "none.json"), *ARGS, _lib(tmp_path))
    assert t is None and "unreadable" in src["reason"]
