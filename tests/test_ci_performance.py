"""The perf-regression script's parsing and verdict (scripts/ci_performance.py); no GPU, no bench run."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("ci_performance", os.path.join(ROOT, "scripts", "ci_performance.py"))
ci = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ci)


def _line(value, gemm, attn, moe, ms):
    return json.dumps(dict(metric="m", value=value, unit="TFLOPS", gemm_tflops=gemm, attn_tflops=attn,
                           moe_tflops_per_gpu=moe, ms_per_step=ms))


def test_parse_takes_the_json_line():
    out = "warning: something\n" + _line(900.0, 1200, 1000, 700, 1.0) + "\n"
    assert ci.parse_bench(out)["gemm_tflops"] == 1200


def test_regression_verdict():
    base = ci.summarize([json.loads(_line(900, 1200, 1000, 700, 1.0)), json.loads(_line(910, 1210, 1010, 690, 0.99))])
    assert base["value"] == 905
    cur_ok = ci.summarize([json.loads(_line(902, 1190, 1020, 700, 0.995))])
    rows, reg = ci.compare(base, cur_ok, 3.0)
    assert reg == [] and len(rows) == 5
    cur_bad = ci.summarize([json.loads(_line(850, 1100, 1000, 700, 1.06))])
    _, reg = ci.compare(base, cur_bad, 3.0)
    assert reg == ["value", "gemm_tflops"]
    assert "gemm_tflops" in ci.format_table(rows)
