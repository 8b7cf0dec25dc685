"""Prints the headline and check fields of the bench JSON line(s) in the given log files (the last `{...}` line of
each): python scripts/line_summary.py gpurun_out/b.log [...]"""
import json
import sys

KEYS = ("value", "n_gpus", "checks_passed", "sgemm_fp32_via_bf16x6_tflops", "reduce_weak_gbps", "reduce_strong_gbps",
        "scan_weak_gbps", "scan_strong_gbps", "stencil_glups", "stencil_halo_mult", "stencil_halo_selftest_bit_exact",
        "stencil_timed_grid_bit_exact", "spmv_gflops", "spmv_pipeline_selftest_bit_identical",
        "spmv_iterated_max_rel_err_vs_fp64", "spmv_max_rel_err_vs_fp64", "rocsparse_spmv_gflops",
        "allreduce_busbw_gbps")


def main():
    for path in sys.argv[1:]:
        lines = [ln for ln in open(path, errors="replace") if ln.startswith("{")]
        if not lines:
            print(f"{path}: no JSON line")
            continue
        d = json.loads(lines[-1])
        picked = {k: d[k] for k in KEYS if k in d}
        picked.update({k: v for k, v in d.items() if "error" in k and "rel_err" not in k or "failed" in k})
        print(f"{path}: {json.dumps(picked)}")


if __name__ == "__main__":
    main()
