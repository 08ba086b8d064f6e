"""The byte / rate models of bench.py's N > 1 lines (round 5): the per-block algorithmic
bytes of a copy_u_sum, the exchange summary against the xGMI links a rank
uses, and the job-level roofline aggregation (every rank's bytes over the slowest rank's
time against N x the HBM peak).  Pure host arithmetic on hand-made records."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class _Csr:
    def __init__(self, rows, nnz):
        self.num_rows, self.nnz = rows, nnz


class _G:
    def __init__(self, rows, nnz):
        self.in_csr = _Csr(rows, nnz)


def test_spmm_alg_bytes():
    assert bench.spmm_alg_bytes(None, 64) == 0
    g = _G(10, 100)
    # indptr + indices + one 256-B row per edge + one 256-B output row per destination
    assert bench.spmm_alg_bytes(g, 64) == 4 * 11 + 4 * 100 + 256 * 100 + 256 * 10
    # the epilogue's addend adds one more row per destination
    assert bench.spmm_alg_bytes(g, 64, addend=True) == bench.spmm_alg_bytes(g, 64) + 256 * 10


def test_exchange_summary_rates_and_links():
    per = [{"bytes_received": 2e9, "bytes_sent": 1e9, "exchange_ms": 10.0},
           {"bytes_received": 1e9, "bytes_sent": 2e9, "exchange_ms": 20.0}]
    agg = bench.exchange_summary(per, 2)
    # rank 0: 2 GB in over 10 ms = 200 GB/s in, 100 GB/s out; one link at N = 2
    assert per[0]["exchange_in_GBps"] == pytest.approx(200.0)
    assert per[0]["exchange_out_GBps"] == pytest.approx(100.0)
    assert per[0]["xgmi_peak_GBps"] == pytest.approx(bench.XGMI_LINK_GBPS)
    assert per[0]["exchange_frac"] == pytest.approx(200.0 / bench.XGMI_LINK_GBPS)
    assert per[1]["exchange_frac"] == pytest.approx(100.0 / bench.XGMI_LINK_GBPS)
    # aggregate: bytes that crossed once (at the receivers) over the slowest exchange
    assert agg["bytes_all_ranks"] == pytest.approx(3e9)
    assert agg["max_exchange_ms"] == pytest.approx(20.0)
    assert agg["GBps"] == pytest.approx(150.0)
    assert agg["peak_GBps"] == pytest.approx(2 * 1 * bench.XGMI_LINK_GBPS)
    assert agg["frac"] == pytest.approx(150.0 / (2 * bench.XGMI_LINK_GBPS))


def test_exchange_summary_eight_ranks_use_seven_links():
    per = [{"bytes_received": 7e8, "bytes_sent": 7e8, "exchange_ms": 1.0} for _ in range(8)]
    agg = bench.exchange_summary(per, 8)
    assert per[3]["xgmi_peak_GBps"] == pytest.approx(7 * bench.XGMI_LINK_GBPS)
    assert agg["peak_GBps"] == pytest.approx(8 * 7 * bench.XGMI_LINK_GBPS)
    assert agg["GBps"] == pytest.approx(8 * 700.0)


def test_exchange_summary_without_time():
    per = [{"bytes_received": 0, "bytes_sent": 0, "exchange_ms": 0.0}]
    agg = bench.exchange_summary(per, 1)
    assert per[0]["exchange_frac"] is None and agg["GBps"] is None and agg["frac"] is None


def _rec(rank, ms, alg, traffic):
    r = {"rank": rank, "kernel_ms": ms, "alg_bytes": alg, "compulsory_bytes": alg // 4,
         "traffic": traffic}
    r["frac"] = alg / (ms * 1e-3) / 1e9 / bench.HBM_PEAK_GBPS
    return r


def test_job_roofline_one_rank_is_the_launch():
    """achieved = the contract's algorithmic bytes / kernel time; the counter bytes
    (L2 egress: HBM + Infinity Cache) and the compulsory bytes bound the HBM fraction."""
    roof, egress = bench.job_roofline([_rec(0, 2.0, 30e9, 16e9)], 1)
    assert roof["achieved"] == pytest.approx(15000.0)
    assert roof["frac"] == pytest.approx(15000.0 / bench.HBM_PEAK_GBPS)
    assert egress == pytest.approx(8000.0) and roof["l2_egress_GBps"] == pytest.approx(8000.0)
    assert roof["l2_egress_frac"] == pytest.approx(1.0)
    assert roof["compulsory_GBps"] == pytest.approx(30e9 // 4 / 2e-3 / 1e9)
    assert roof["hbm_frac_bounds"] == pytest.approx([roof["compulsory_frac"], 1.0])
    assert roof["peak"] == bench.HBM_PEAK_GBPS and roof["traffic"] == 16e9
    assert "per_rank" not in roof


def test_job_roofline_aggregates_over_the_slowest_rank():
    per = [_rec(0, 2.0, 30e9, 14e9), _rec(1, 2.5, 30e9, 16e9)]
    roof, egress = bench.job_roofline(per, 2)
    # every rank's bytes over the slowest 2.5 ms against 2 x 8 TB/s -- not the best rank's
    assert roof["achieved"] == pytest.approx(60e9 / 2.5e-3 / 1e9)
    assert roof["frac"] == pytest.approx(24000.0 / 16000.0)
    assert egress == pytest.approx(30e9 / 2.5e-3 / 1e9)
    assert roof["l2_egress_frac"] == pytest.approx(12000.0 / 16000.0)
    assert roof["peak"] == pytest.approx(2 * bench.HBM_PEAK_GBPS)
    assert roof["frac_min"] == pytest.approx(per[1]["frac"])
    assert roof["alg_bytes_per_launch"] == pytest.approx(60e9)
    assert roof["alg_GBps"] == pytest.approx(60e9 / 2.5e-3 / 1e9)
    # a rank without counters: the algorithmic figure stays, no counter-based one
    roof2, eg2 = bench.job_roofline([_rec(0, 2.0, 30e9, 14e9), _rec(1, 2.0, 30e9, None)], 2)
    assert eg2 is None and roof2["traffic"] is None and roof2["hbm_frac_bounds"] is None
    assert roof2["frac"] == pytest.approx(30000.0 / 16000.0)
