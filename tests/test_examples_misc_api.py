"""Small API examples: quickstart, compile flags, layout visualisation, MFMA layout plots, lazy_jit."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("", "compile_flags", "visual_layout_inference", "plot_layout", "lazy_jit"):
    sys.path.insert(0, os.path.join(ROOT, "examples", d))

import tilelang  # noqa: E402


def test_quickstart_cpu():
    import quickstart
    quickstart.main(128, 128, 128, cpu=True)


def test_compile_flags_reach_the_device_compiler():
    import usecase
    k = usecase.build(256, 256, 256, target="hip", flags=("-O3", "-ffast-math"))
    assert "-ffast-math" in k.compile_flags and len(k.code[0]) > 0
    k2 = usecase.build(256, 256, 256, target="hip", flags=("-O2", ))
    assert k2 is not k  # flags are part of the cache key


def test_layout_visualization_dump(tmp_path, monkeypatch):
    monkeypatch.setenv("TILELANG_LAYOUT_DIR", str(tmp_path))
    import visual_layout_inference as v
    f = v.matmul.get_tir(128, 128, 128, 32, 32, 32)
    tilelang.compile(f, out_idx=[-1], target="hip", pass_configs=v.matmul.pass_configs)
    files = os.listdir(tmp_path)
    assert any(x.endswith(".layouts.txt") for x in files) and any(x.endswith(".svg") for x in files)
    txt = open(os.path.join(tmp_path, [x for x in files if x.endswith(".layouts.txt")][0])).read()
    assert "C_local" in txt


def test_plot_mfma_layouts(tmp_path):
    import fragment_mfma_load_a as p
    a = p.make_mfma_load_base_layout("float16", "A")
    # lane l holds A[l % 16][8 * (l // 16) + j]
    from tilelang.tools.plot_layout import layout_grid
    g = layout_grid(a)
    assert g[3][0] == (3, 0) and g[0][8] == (16, 0) and g[5][13] == (21, 5)
    c = p.make_mfma_store_layout()
    assert layout_grid(c)[5][2] == (18, 1)  # C[4 * (l // 16) + v][l % 16]
    p.main(str(tmp_path))
    assert any(x.endswith(".svg") for x in os.listdir(tmp_path))


def test_lazy_jit_walkthrough_cpu():
    import lazyjit
    lazyjit.main("cpu")


@pytest.mark.gpu
def test_small_api_examples_gpu():
    import quickstart
    import usecase
    import lazyjit
    quickstart.main(512, 512, 512)
    usecase.main()
    lazyjit.main("cuda")
