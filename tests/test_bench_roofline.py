"""bench.py's roofline fields from the PMC table (host logic, CPU): a PMC
entry collected on other kernel sources is reported as stale and its
counter-derived fields are omitted; a current one yields traffic, VALU,
fabric and texture-data-path fractions."""
import importlib.util
import os

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _pmc(sha):
    return {"source": "x", "kernel_sources_sha": sha, "hbm_bytes_per_launch": 8e10,
            "valu_insts_per_launch": 5.6e9, "fabric_ceiling_lines_per_s": 5.0e10,
            "hbm_gather_ceiling_lines_per_s": 4.5e10,
            "counters_per_launch": {"TCC_MISS_sum": 6.0e8, "TCC_HIT_sum": 1.2e9, "GRBM_GUI_ACTIVE": 2.4e8,
                                    "SQ_INSTS_VMEM_RD": 2.1e8, "TD_TD_BUSY_sum": 7.5e9}}


def test_sources_sha_is_stable_and_covers_the_kernels():
    b = _bench()
    assert b.kernel_sources_sha() == b.kernel_sources_sha()
    assert len(b.kernel_sources_sha()) == 16
    assert "sc_windows.hip" in b.KERNEL_SOURCES and "sc_device.hpp" in b.KERNEL_SOURCES


def test_current_pmc_gives_td_and_fabric_fractions():
    b = _bench()
    r = b.roofline(300.0, 8e10, 5.6e9, 0.0135, 4.2e9, 4.3e9, 0.0138, _pmc(b.kernel_sources_sha()), {}, 30)
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
