"""bench.py's roofline fields from the PMC table (host logic, CPU): a PMC
entry collected on another build (sc_build_info build_id) is reported as
stale and its counter-derived fields are omitted; a current one yields
traffic, VALU, fabric and texture-data-path fractions (VERDICT r3 weak #7,
r4 next #6)."""
import importlib.util
import os

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _pmc(bid):
    return {"source": "x", "build_id": bid, "hbm_bytes_per_launch": 8e10,
            "valu_insts_per_launch": 5.6e9, "fabric_ceiling_lines_per_s": 5.0e10,
            "hbm_gather_ceiling_lines_per_s": 4.5e10,
            "counters_per_launch": {"TCC_MISS_sum": 6.0e8, "TCC_HIT_sum": 1.2e9, "GRBM_GUI_ACTIVE": 2.4e8,
                                    "SQ_INSTS_VMEM_RD": 2.1e8, "TD_TD_BUSY_sum": 7.5e9}}


def test_build_id_covers_every_source_and_flag(tmp_path, monkeypatch):
    """The id changes with the launch schedule (sc_api.cpp), the kernels, the
    Makefile and the -D flags; a PMC entry of another id is stale."""
    import shutil
    b = _bench()
    bid = b.source_build_id()
    assert bid == b.source_build_id() and len(bid) == 16
    assert b.source_build_id("-DSC_CHAIN_BATCH=64") != bid
    csrc = tmp_path / "csrc"
    shutil.copytree(b.CSRC, csrc, ignore=shutil.ignore_patterns("*.o", "*.so"))
    monkeypatch.setattr(b, "CSRC", str(csrc))
    assert b.source_build_id() == bid
    for f in ("sc_api.cpp", "sc_windows.hip", "Makefile"):
        p = csrc / f
        old = p.read_bytes()
        p.write_bytes(old + b"\n// a schedule change\n")
        assert b.source_build_id() != bid, f
        p.write_bytes(old)
    assert not b.pmc_is_stale(_pmc(bid), bid)
    assert b.pmc_is_stale(_pmc(bid), b.source_build_id("-DX=1"))
    assert not b.pmc_is_stale({}, bid)


def test_current_pmc_gives_td_and_fabric_fractions():
    b = _bench()
    r = b.roofline(300.0, 8e10, 5.6e9, 0.0135, 4.2e9, 4.3e9, 0.0138, _pmc(b.source_build_id()), {}, 30)
    assert "pmc_stale" not in r
    cyc = 2.4e8 / 8
    assert abs(r["td_frac"] - 2.1e8 * 16 / (256 * cyc)) < 1e-12
    assert abs(r["td_busy_frac"] - 7.5e9 / (256 * cyc)) < 1e-12
    assert abs(r["fabric_frac"] - 6.0e8 / 0.0135 / 5.0e10) < 1e-12
    assert abs(r["l2_hit"] - 1.2 / 1.8) < 1e-12


def test_stale_pmc_is_reported_not_used():
    b = _bench()
    stale = {"source": "x", "stale": True}
    r = b.roofline(300.0, None, None, 0.0135, 4.2e9, 4.3e9, 0.0138, stale, {}, 30)
    assert "pmc_stale" in r
    for k in ("fabric_frac", "td_frac", "td_busy_frac", "l2_hit"):
        assert k not in r
    assert r["traffic"] is None and r["valu"] is None
