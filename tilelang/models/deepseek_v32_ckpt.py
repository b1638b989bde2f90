"""DeepSeek-V3.2 checkpoints: HF safetensors -> per-rank shards -> ``Transformer`` parameters.

Reference: ``examples/deepseek_v32/inference/convert.py`` (HF names -> ``model{rank}-mp{ws}``
shards: column-parallel weights split on dim 0, row-parallel on dim 1, routed experts dealt out
whole, the rest replicated) and ``generate.py:119`` (``load_model`` of the rank's shard).

* ``convert(hf_dir, save_dir, n_experts, mp)`` -- streams every ``*.safetensors`` of ``hf_dir``
  (safetensors ``safe_open``: nothing is unpickled), renames with the reference's key map and
  writes one shard per rank; fp8 e4m3 weights keep their ``weight_scale_inv`` (renamed ``scale``,
  one fp32 per 128x128 block) and the scale is split with its weight.  Tokenizer files are copied.
* ``load_model(model, path)`` -- fills a ``Transformer`` built for the same world size from its
  rank's shard.  Name translation to this implementation's modules: ``ffn.experts.{e}.w1/w3``
  (gate / up) are packed into the grouped-GEMM ``[n_local, 2F, H]`` table, ``ffn.experts.{e}.w2``
  into ``[n_local, H, F]``, ``ffn.shared_experts`` is ``ffn.shared``.  Precision follows the model:
  an fp8 tensor loaded into a bf16 parameter is dequantised (``weight_dequant``), a bf16 tensor
  loaded into an fp8 projection is block-quantised (``weight_quant``).  Every parameter must be
  covered (strict), so a wrong shard never leaves random weights behind.
* ``export_hf(model, out_dir)`` -- the inverse naming, for a world-size-1 model: writes the model
  as an HF-style checkpoint (tests round-trip synthetic weights through convert -> load).
"""
from __future__ import annotations

import os
import shutil
from glob import glob
from typing import Dict, Optional

import torch

# HF module name -> (reference module name, split dim for model parallelism or None)
KEY_MAP = {
    "embed_tokens": ("embed", 0),
    "input_layernorm": ("attn_norm", None),
    "post_attention_layernorm": ("ffn_norm", None),
    "q_proj": ("wq", 0),
    "q_a_proj": ("wq_a", None),
    "q_a_layernorm": ("q_norm", None),
    "q_b_proj": ("wq_b", 0),
    "kv_a_proj_with_mqa": ("wkv_a", None),
    "kv_a_layernorm": ("kv_norm", None),
    "kv_b_proj": ("wkv_b", 0),
    "o_proj": ("wo", 1),
    "gate": ("gate", None),
    "gate_proj": ("w1", 0),
    "down_proj": ("w2", 1),
    "up_proj": ("w3", 0),
    "norm": ("norm", None),
    "lm_head": ("head", 0),
    "scale": ("scale", None),
    # the DSA indexer's projections keep their names and are replicated
    "wq_b": ("wq_b", None),
    "wk": ("wk", None),
    "k_norm": ("k_norm", None),
    "weights_proj": ("weights_proj", None),
}


def _rename(name: str):
    """HF tensor name -> (reference name, split dim)."""
    if name.startswith("model."):
        name = name[len("model."):]
    name = name.replace("self_attn", "attn").replace("mlp", "ffn")
    name = name.replace("weight_scale_inv", "scale").replace("e_score_correction_bias", "bias")
    parts = name.split(".")
    key = parts[-2]
    if key not in KEY_MAP:
        raise KeyError(f"unknown checkpoint tensor {name!r} (module {key!r})")
    new, dim = KEY_MAP[key]
    parts[-2] = new
    return ".".join(parts), dim


def _expert_index(name: str) -> Optional[int]:
    parts = name.split(".")
    if "experts" in parts and "shared_experts" not in name:
        return int(parts[parts.index("experts") + 1])
    return None


def convert(hf_dir: str, save_dir: str, n_experts: int, mp: int, skip_layers=("layers.61", )) -> list:
    """HF safetensors -> ``model{i}-mp{mp}.safetensors`` for i < mp; returns the shard paths.
    ``skip_layers``: name fragments to drop (the reference drops the MTP layer 61)."""
    from safetensors import safe_open
    from safetensors.torch import save_file
    if n_experts % mp:
        raise ValueError(f"{n_experts} experts do not split over {mp} ranks")
    n_local = n_experts // mp
    shards: list = [{} for _ in range(mp)]
    files = sorted(glob(os.path.join(hf_dir, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no *.safetensors in {hf_dir}")
    for path in files:
        with safe_open(path, framework="pt", device="cpu") as f:
            for hf_name in f.keys():
                if any(s in hf_name for s in skip_layers):
                    continue
                t = f.get_tensor(hf_name)
                name, dim = _rename(hf_name)
                e = _expert_index(name)
                for i in range(mp):
                    if e is not None:
                        if not (i * n_local <= e < (i + 1) * n_local):
                            continue
                        shards[i][name] = t
                    elif dim is not None:
                        if t.size(dim) % mp:
                            raise ValueError(f"{hf_name}: dim {dim} of size {t.size(dim)} does not split over {mp}")
                        n = t.size(dim) // mp
                        shards[i][name] = t.narrow(dim, i * n, n).contiguous()
                    else:
                        shards[i][name] = t
    os.makedirs(save_dir, exist_ok=True)
    out = []
    for i in range(mp):
        p = os.path.join(save_dir, f"model{i}-mp{mp}.safetensors")
        save_file(shards[i], p)
        out.append(p)
    for p in glob(os.path.join(hf_dir, "*token*")):
        shutil.copyfile(p, os.path.join(save_dir, os.path.basename(p)))
    return out


# ---- loading ----------------------------------------------------------------------------------

def _dequant(w: torch.Tensor, s: torch.Tensor, dtype) -> torch.Tensor:
    from ..ops.fp8_gemm import weight_dequant
    return weight_dequant(w, s.float()).to(dtype)


def _as_param(param: torch.nn.Parameter, t: torch.Tensor, what: str):
    if tuple(param.shape) != tuple(t.shape):
        raise ValueError(f"{what}: checkpoint shape {tuple(t.shape)} != model shape {tuple(param.shape)}")
    with torch.no_grad():
        param.copy_(t.to(param.dtype))


def load_model(model, path: str, strict: bool = True) -> Dict[str, int]:
    """Fill ``model`` (a ``deepseek_v32.Transformer`` built for this rank's world size) from the
    shard at ``path``.  Returns {"tensors": n, "params": n}."""
    from safetensors import safe_open
    from . import deepseek_v32 as D
    with safe_open(path, framework="pt", device="cpu") as f:
        sd = {k: f.get_tensor(k) for k in f.keys()}
    params = dict(model.named_parameters())
    done = set()
    used = set()

    def take(name):
        used.add(name)
        return sd[name]

    # 1. every Linear (possibly fp8 + scale) and plain parameter, by name
    for mod_name, mod in model.named_modules():
        if isinstance(mod, D.Linear):
            wname = f"{mod_name}.weight"
            if wname not in sd:
                continue
            w = take(wname)
            s = take(f"{mod_name}.scale") if f"{mod_name}.scale" in sd else None
            if mod.scale is not None:  # the model keeps this projection in fp8
                if s is None:
                    from ..ops.fp8_gemm import weight_quant
                    w, s = weight_quant(w.to(mod.out_dtype).contiguous())
                _as_param(mod.weight, w.to(mod.weight.dtype), wname)
                _as_param(mod.scale, s.float(), f"{mod_name}.scale")
                done.update({wname, f"{mod_name}.scale"})
            else:
                if s is not None:
                    w = _dequant(w, s, mod.weight.dtype)
                _as_param(mod.weight, w, wname)
                done.add(wname)
            if isinstance(mod, D.Linear) and mod_name.endswith("attn.wkv_b"):
                parent = model.get_submodule(mod_name.rsplit(".", 1)[0])
                parent._absorb = None  # the absorbed projections are derived from wkv_b
    # 2. routed experts: per-expert w1/w3/w2 -> the packed grouped-GEMM tables
    for mod_name, mod in model.named_modules():
        if not isinstance(mod, D.MoE):
            continue
        F = mod.w2.shape[-1]
        for el in range(mod.n_local):
            e = mod.first + el
            pre = f"{mod_name}.experts.{e}"
            ws = {}
            for k in ("w1", "w2", "w3"):
                wn = f"{pre}.{k}.weight"
                if wn not in sd:
                    if strict:
                        raise KeyError(f"checkpoint misses {wn}")
                    continue
                w = take(wn)
                sn = f"{pre}.{k}.scale"
                if sn in sd:
                    w = _dequant(w, take(sn), mod.w1.dtype)
                ws[k] = w.to(mod.w1.dtype)
            with torch.no_grad():
                if "w1" in ws:
                    mod.w1[el, :F].copy_(ws["w1"])
                if "w3" in ws:
                    mod.w1[el, F:].copy_(ws["w3"])
                if "w2" in ws:
                    mod.w2[el].copy_(ws["w2"])
        done.update({f"{mod_name}.w1", f"{mod_name}.w2"})
    # 3. the shared experts are named ``shared`` here, ``shared_experts`` in the checkpoint
    alias = {}
    for n in sd:
        if ".ffn.shared_experts." in n:
            alias[n.replace(".ffn.shared_experts.", ".ffn.shared.")] = n
    for mod_name, mod in model.named_modules():
        if isinstance(mod, D.Linear) and ".ffn.shared." in mod_name:
            wname = f"{mod_name}.weight"
            src = alias.get(wname)
            if src is None:
                continue
            w = take(src)
            s_src = src[:-len(".weight")] + ".scale"
            s = take(s_src) if s_src in sd else None
            if mod.scale is not None:
                if s is None:
                    from ..ops.fp8_gemm import weight_quant
                    w, s = weight_quant(w.to(mod.out_dtype).contiguous())
                _as_param(mod.weight, w.to(mod.weight.dtype), wname)
                _as_param(mod.scale, s.float(), f"{mod_name}.scale")
                done.update({wname, f"{mod_name}.scale"})
            else:
                if s is not None:
                    w = _dequant(w, s, mod.weight.dtype)
                _as_param(mod.weight, w, wname)
                done.add(wname)
    # 4. everything else that is a plain parameter of the same name (norms, gate, embedding)
    for name, p in params.items():
        if name in done or name not in sd:
            continue
        _as_param(p, take(name), name)
        done.add(name)
    if strict:
        missing = sorted(set(params) - done)
        unused = sorted(set(sd) - used)
        if missing:
            raise KeyError(f"{path}: no checkpoint tensor for {missing[:8]}{' ...' if len(missing) > 8 else ''}")
        if unused:
            raise KeyError(f"{path}: checkpoint tensors with no parameter: {unused[:8]}")
    return {"tensors": len(used), "params": len(done)}


# ---- export (tests, world size 1) -------------------------------------------------------------

_REF_TO_HF = {
    "embed": "embed_tokens", "attn_norm": "input_layernorm", "ffn_norm": "post_attention_layernorm",
    "wq_a": "q_a_proj", "q_norm": "q_a_layernorm", "wkv_a": "kv_a_proj_with_mqa", "kv_norm": "kv_a_layernorm",
    "wkv_b": "kv_b_proj", "wo": "o_proj", "norm": "norm", "head": "lm_head", "gate": "gate",
    "w1": "gate_proj", "w2": "down_proj", "w3": "up_proj",
}


def _hf_name(ref_name: str) -> str:
    parts = ref_name.split(".")
    is_scale = parts[-1] == "scale"
    mod = parts[-2]
    indexer = "indexer" in parts
    if mod == "wq_b":
        mod = "wq_b" if indexer else "q_b_proj"
    elif not indexer:
        mod = _REF_TO_HF.get(mod, mod)
    parts[-2] = mod
    if is_scale:
        parts[-1] = "weight_scale_inv"
    if parts[-1] == "bias" and mod == "gate":
        parts[-1] = "e_score_correction_bias"
    name = ".".join(parts).replace(".attn.", ".self_attn.").replace(".ffn.", ".mlp.")
    if name.startswith("head.") or name.startswith("lm_head."):
        return name.replace("head.", "lm_head.", 1) if name.startswith("head.") else name
    return "model." + name


def export_hf(model, out_dir: str, shard_size: int = 64) -> list:
    """Write a world-size-1 ``Transformer`` as HF-named safetensors (fp8 projections keep their
    ``weight_scale_inv``); ``shard_size`` tensors per file, like a multi-file HF checkpoint."""
    from safetensors.torch import save_file
    from . import deepseek_v32 as D
    ref: Dict[str, torch.Tensor] = {}
    for mod_name, mod in model.named_modules():
        if isinstance(mod, D.MoE):
            F = mod.w2.shape[-1]
            for el in range(mod.n_local):
                e = mod.first + el
                ref[f"{mod_name}.experts.{e}.w1.weight"] = mod.w1[el, :F]
                ref[f"{mod_name}.experts.{e}.w3.weight"] = mod.w1[el, F:]
                ref[f"{mod_name}.experts.{e}.w2.weight"] = mod.w2[el]
    for name, p in model.named_parameters():
        if name.endswith(".ffn.w1") or name.endswith(".ffn.w2"):
            continue
        ref[name.replace(".ffn.shared.", ".ffn.shared_experts.")] = p
    hf = {_hf_name(k): v.detach().cpu().contiguous() for k, v in ref.items()}
    os.makedirs(out_dir, exist_ok=True)
    names = sorted(hf)
    out = []
    for i in range(0, len(names), shard_size):
        p = os.path.join(out_dir, f"model-{i // shard_size:05d}.safetensors")
        save_file({k: hf[k] for k in names[i:i + shard_size]}, p)
        out.append(p)
    return out
