"""Machine-readable result lines (one JSON object per line on stdout) and the bench-line contract.

`bench_line` builds the ONE line bench.py prints on rank 0 and checks it against the contract the round driver
parses: the required keys and their types, `value` = whole-job aggregate (sum over the N GPUs), `n_gpus` = N,
`vs_baseline` = value / the BASELINE.md number (None when the reference publishes none, as here:
BASELINE.json "published": {}), and the config block naming the BASELINE.json model/config. A malformed line raises
instead of being printed, so a contract slip fails the bench run (and tests/test_metrics.py) rather than the
driver's parser.
"""
from __future__ import annotations

import json
import math
import sys

# key -> accepted types of the driver's bench-line contract
BENCH_KEYS = {
    "metric": (str,), "value": (int, float), "unit": (str,), "n_gpus": (int,), "steps": (int,), "warmup": (int,),
    "ms_per_step": (int, float), "higher_is_better": (bool,), "scaling": (str,), "vs_baseline": (int, float, type(None)),
    "dtype": (str,), "data": (str,), "config": (dict,),
}
CONFIG_KEYS = ("model", "global_batch", "seq_len", "parallelism")


def emit_metric(stream=None, **fields) -> dict:
    line = json.dumps(fields, default=str)
    print(line, file=stream or sys.stdout, flush=True)
    return fields


def validate_bench_line(line: dict, partial: bool = False) -> dict:
    """Raises ValueError naming every contract violation of a bench line; returns the line. partial=True (a lab run
    of some sections without the headline one) lets value / ms_per_step be null."""
    bad = []
    for k, types in BENCH_KEYS.items():
        if k not in line:
            bad.append(f"missing {k}")
        elif partial and k in ("value", "ms_per_step") and line[k] is None:
            continue
        elif not isinstance(line[k], types) or (isinstance(line[k], bool) and bool not in types):
            bad.append(f"{k}: {type(line[k]).__name__}")
    if not bad:
        if line["value"] is not None and (not math.isfinite(line["value"]) or line["value"] < 0):
            bad.append(f"value {line['value']}")
        if line["scaling"] not in ("weak", "strong"):
            bad.append(f"scaling {line['scaling']!r}")
        if line["n_gpus"] < 1 or line["steps"] < 1 or line["warmup"] < 0:
            bad.append("n_gpus / steps / warmup out of range")
        bad += [f"config missing {k}" for k in CONFIG_KEYS if k not in line["config"]]
    if bad:
        raise ValueError("bench line violates the driver contract: " + "; ".join(bad))
    return line


def bench_line(*, metric: str, value: float, unit: str, n_gpus: int, steps: int, warmup: int, ms_per_step: float,
               dtype: str, data: str, config: dict, baseline: float | None = None, higher_is_better: bool = True,
               scaling: str = "weak", partial: bool = False, **extra) -> dict:
    """The validated bench line: contract keys first (vs_baseline = value / baseline when a baseline number exists),
    then the extra per-section fields in insertion order."""
    vs = None if baseline in (None, 0) or value is None else value / baseline
    line = {"metric": metric, "value": value, "unit": unit, "n_gpus": n_gpus, "steps": steps, "warmup": warmup,
            "ms_per_step": ms_per_step, "higher_is_better": higher_is_better, "scaling": scaling, "vs_baseline": vs,
            "dtype": dtype, "data": data, "config": config}
    clash = set(extra) & set(line)
    if clash:
        raise ValueError(f"extra fields shadow contract keys: {sorted(clash)}")
    line.update(extra)
    return validate_bench_line(line, partial)
