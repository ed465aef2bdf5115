"""The measurement arithmetic behind roofline.traffic and the committed records (CPU only):
tools/prof_summary.py's traffic (FETCH_SIZE x2 + WRITE_SIZE, KB -> B, per order of the run, the
config-4 seeding batches dropped with --from-sweep) and dram (32-B request units) summaries on
synthetic rocprofv3 counter CSVs, and the committed closing record's internal consistency (the
per-kernel bytes add up to the total; profiles/INDEX.md names the build the traffic file carries)."""
import csv
import importlib.util
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ps():
    spec = importlib.util.spec_from_file_location("prof_summary", os.path.join(ROOT, "tools", "prof_summary.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _csv(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "pmc_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for did, kern, cn, v in rows:
            w.writerow({"Dispatch_Id": did, "Kernel_Name": kern, "Counter_Name": cn, "Counter_Value": v})


def _bench_log(path, steps, warmup, batch):
    line = {"metric": "m", "steps": steps, "warmup": warmup, "build": "src=test",
            "config": {"global_batch": batch, "workload": "w"}}
    with open(path, "w") as f:
        f.write("some stderr noise\n" + json.dumps(line) + "\n")


def test_traffic_bytes_per_order(ps, tmp_path, capsys):
    # two dispatches of a walk, one of a side kernel; FETCH_SIZE / WRITE_SIZE in KB, summed over XCD rows
    fetch = [(1, "void k_walk(A)", "FETCH_SIZE", 10.0), (1, "void k_walk(A)", "FETCH_SIZE", 6.0),
             (2, "void k_walk(A)", "FETCH_SIZE", 4.0), (3, "me::k_side(B)", "FETCH_SIZE", 5.0)]
    write = [(1, "void k_walk(A)", "WRITE_SIZE", 3.0), (2, "void k_walk(A)", "WRITE_SIZE", 1.0),
             (3, "me::k_side(B)", "WRITE_SIZE", 8.0)]
    _csv(str(tmp_path / "f"), fetch)
    _csv(str(tmp_path / "w"), write)
    _bench_log(str(tmp_path / "b.log"), steps=3, warmup=1, batch=256)
    ps.traffic(str(tmp_path / "f"), str(tmp_path / "w"), str(tmp_path / "b.log"))
    out = json.loads(capsys.readouterr().out)
    orders = 4 * 256
    assert out["orders"] == orders
    walk = out["per_kernel"]["k_walk"]
    assert walk["dispatches"] == 2
    assert walk["fetch_bytes_per_order"] == pytest.approx(2 * 1024 * 20.0 / orders)  # x2 gfx950 correction
    assert walk["write_bytes_per_order"] == pytest.approx(1024 * 4.0 / orders)
    tot = 2 * 1024 * 25.0 + 1024 * 12.0
    assert out["bytes_per_order"] == pytest.approx(tot / orders)
    assert out["build"] == "src=test"


def test_traffic_from_sweep_drops_seeding(ps, tmp_path, capsys):
    # dispatch ids ascend; sweeps at 1, 4, 7: --from-sweep 1 keeps dispatches >= 4 only
    rows_f, rows_w = [], []
    for did, kern in [(1, "me::k_seq_sweep(X)"), (2, "k_match(Y)"), (3, "k_match(Y)"), (4, "me::k_seq_sweep(X)"),
                      (5, "k_match(Y)"), (7, "me::k_seq_sweep(X)"), (8, "k_match(Y)")]:
        rows_f.append((did, kern, "FETCH_SIZE", 1.0))
        rows_w.append((did, kern, "WRITE_SIZE", 1.0))
    _csv(str(tmp_path / "f"), rows_f)
    _csv(str(tmp_path / "w"), rows_w)
    _bench_log(str(tmp_path / "b.log"), steps=1, warmup=0, batch=1024)
    ps.traffic(str(tmp_path / "f"), str(tmp_path / "w"), str(tmp_path / "b.log"), from_sweep=1)
    out = json.loads(capsys.readouterr().out)
    assert out["from_sweep"] == 1
    assert out["per_kernel"]["k_match"]["dispatches"] == 2  # dispatches 5 and 8
    assert out["per_kernel"]["me::k_seq_sweep"]["dispatches"] == 2  # 4 and 7
    assert out["bytes_per_order"] == pytest.approx((2 * 1024 * 4 + 1024 * 4) / 1024)


def test_dram_32b_units(ps, tmp_path, capsys):
    rows = [(1, "k_agg(Z)", "TCC_EA0_RDREQ_DRAM_32B", 400.0), (1, "k_agg(Z)", "TCC_EA0_WRREQ_WRITE_DRAM_32B", 100.0),
            (1, "k_agg(Z)", "TCC_EA0_WRREQ_WRITE_ATOMIC_32B", 10.0), (1, "k_agg(Z)", "TCC_EA0_RDREQ", 100.0)]
    _csv(str(tmp_path / "d"), rows)
    _bench_log(str(tmp_path / "b.log"), steps=1, warmup=0, batch=32)
    ps.dram(str(tmp_path / "d"), str(tmp_path / "b.log"))
    out = json.loads(capsys.readouterr().out)
    k = out["per_kernel"]["k_agg"]
    assert k["read_bytes_per_order"] == pytest.approx(32 * 400.0 / 32)
    assert k["mean_read_request_bytes"] == pytest.approx(128.0)  # four 32-B units per request
    assert out["bytes_per_order"] == pytest.approx(32 * 510.0 / 32)


def test_committed_traffic_record_consistent():
    """profiles/pmc_traffic.json (bench.py's roofline.traffic source) adds up, and profiles/INDEX.md's
    current closing record names the build it carries."""
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    per = d["per_kernel"].values()
    assert sum(v["bytes_per_order"] for v in per) == pytest.approx(d["bytes_per_order"], rel=1e-9)
    assert d["bytes_per_order"] == pytest.approx(d["fetch_bytes_per_order"] + d["write_bytes_per_order"], rel=1e-9)
    index = open(os.path.join(ROOT, "profiles", "INDEX.md")).read()
    m = re.search(r"## Round \d+ \(current\): closing record `([^`]+)`, build `(src=[0-9a-f]+)`", index)
    assert m, "INDEX.md names no current closing record"
    assert d["build"].startswith(m.group(2)), (d["build"], m.group(2))
    rec = json.load(open(os.path.join(ROOT, "profiles", m.group(1), "pmc_traffic_c2.json")))
    assert rec["bytes_per_order"] == pytest.approx(d["bytes_per_order"])
