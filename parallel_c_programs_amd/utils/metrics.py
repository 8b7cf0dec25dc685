"""Machine-readable benchmark lines (one JSON object per line on stdout)."""
from __future__ import annotations

import json
import sys


def emit_metric(stream=None, **fields) -> dict:
    line = json.dumps(fields, default=str)
    print(line, file=stream or sys.stdout, flush=True)
    return fields
