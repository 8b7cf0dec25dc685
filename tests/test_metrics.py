"""The bench-line contract (utils/metrics.py): what bench.py prints is what the round driver parses."""
import json
import os
import subprocess
import sys

import pytest

from parallel_c_programs_amd.utils.metrics import BENCH_KEYS, bench_line, validate_bench_line

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = {"model": "SGEMM 8192x8192x8192 fp32", "global_batch": 1, "seq_len": None, "parallelism": "dp1"}


def _line(**kw):
    args = dict(metric="m", value=150.0, unit="TFLOPS", n_gpus=1, steps=10, warmup=3, ms_per_step=7.2, dtype="fp32",
                data="synthetic", config=dict(CFG))
    args.update(kw)
    return bench_line(**args)


def test_bench_line_keys_order_and_extras():
    line = _line(sgemm_tflops_per_gpu=150.0)
    assert list(line)[:len(BENCH_KEYS)] == list(BENCH_KEYS)
    assert line["vs_baseline"] is None and line["sgemm_tflops_per_gpu"] == 150.0
    assert _line(baseline=100.0)["vs_baseline"] == pytest.approx(1.5)
    json.dumps(line)


@pytest.mark.parametrize("bad", [dict(value=float("nan")), dict(value=-1.0), dict(scaling="linear"), dict(n_gpus=0),
                                 dict(steps=True), dict(config={"model": "x"}), dict(value=None)])
def test_bench_line_rejects(bad):
    with pytest.raises(ValueError):
        _line(**bad)


def test_bench_line_partial_and_shadowing():
    assert _line(value=None, ms_per_step=None, partial=True)["value"] is None
    with pytest.raises(ValueError, match="shadow"):
        _line(vs_baseline=2.0)  # an extra field may not overwrite a contract key
    with pytest.raises(ValueError, match="missing"):
        validate_bench_line({"metric": "m"})


def test_bench_small_cpu_prints_a_valid_line():
    """bench.py --small on the CPU (one rank): the one JSON line passes the contract check."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--small", "--device", "cpu", "--steps", "1",
                        "--warmup", "0", "--sections", "sgemm,reduce"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    validate_bench_line(line)
    assert line["n_gpus"] == 1 and line["value"] > 0


def test_bench_prints_line_with_contract_error(monkeypatch, capsys):
    """A line that fails the contract is still printed (with the reason) and bench.main returns 1."""
    import importlib

    import parallel_c_programs_amd.utils.metrics as M

    sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")

    def broken(**kw):
        raise ValueError("bench line violates the driver contract: test")

    monkeypatch.setattr(M, "bench_line", broken)
    rc = bench.main(["--small", "--device", "cpu", "--steps", "1", "--warmup", "0", "--sections", "reduce"])
    line = json.loads([ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1])
    assert rc == 1 and "test" in line["contract_error"] and line["vs_baseline"] is None and "reduce_weak_gbps" in line
