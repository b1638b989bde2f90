"""Autotuner (reference ``tilelang/autotuner/{tuner,param,capture}.py``).

``@tilelang.autotune(configs=...)`` wraps a ``@tilelang.jit`` kernel factory.  For a call
with the non-tuned arguments it

  1. compiles every config concurrently (hipcc runs as subprocesses, so a thread pool
     scales; worker count from ``TILELANG_AUTO_TUNING_CPU_COUNTS`` / ``..._MAX_CPU_COUNT``);
     ``compile_backend="process"`` / ``TILELANG_AUTOTUNE_COMPILE=process`` lowers in worker
     processes too (the Python passes are GIL-bound in threads; ``compile_worker.py``),
  2. benchmarks the compiled kernels one at a time on the GPU (L2+MALL flush between
     runs, per-config timeout, optional correctness check against ``ref_prog``) -- on the
     tensors captured by ``set_autotune_inputs`` when a capture is active; with
     ``isolate=True`` (or ``TILELANG_AUTOTUNE_ISOLATE=1``) each config is checked and timed in a
     child process that is killed at the timeout (``autotuner/worker.py``), so a kernel that
     never returns costs one config, not the run,
  3. returns the fastest ``JITKernel`` with ``.config`` / ``.latency`` set, and
  4. persists the winner under ``$TILELANG_CACHE_DIR/autotuner/<sha256>.json`` so the
     next process skips the search.
"""
from __future__ import annotations

import functools
import hashlib
import inspect
import json
import logging
import os
import signal
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Callable, Dict, List, Optional

from ..env import env

logger = logging.getLogger("tilelang.autotuner")


@dataclass
class CompileArgs:
    out_idx: Any = None
    target: str = "auto"
    pass_configs: Optional[dict] = None
    backend: Optional[str] = None  # "thread" | "process"; None: TILELANG_AUTOTUNE_COMPILE (default thread)


@dataclass
class ProfileArgs:
    warmup: int = 25
    rep: int = 100
    timeout: int = 30
    supply_type: Any = None
    ref_prog: Optional[Callable] = None
    supply_prog: Optional[Callable] = None
    rtol: float = 1e-2
    atol: float = 1e-2
    max_mismatched_ratio: float = 0.01
    skip_check: bool = False
    manual_check_prog: Optional[Callable] = None
    cache_input_tensors: bool = True
    isolate: Optional[bool] = None  # None: TILELANG_AUTOTUNE_ISOLATE


@dataclass
class AutotuneResult:
    latency: float = float("inf")
    config: Optional[dict] = None
    ref_latency: Optional[float] = None
    kernel: Any = None
    all_results: List[dict] = field(default_factory=list)

    def save_to_disk(self, path: Path):
        path.parent.mkdir(parents=True, exist_ok=True)
        tmp = path.with_suffix(".tmp")
        tmp.write_text(json.dumps({"latency": self.latency, "config": self.config, "ref_latency": self.ref_latency,
                                   "all": self.all_results}, default=str))
        os.replace(tmp, path)

    @staticmethod
    def load_from_disk(path: Path) -> Optional["AutotuneResult"]:
        if not path.exists():
            return None
        d = json.loads(path.read_text())
        return AutotuneResult(latency=d["latency"], config=d["config"], ref_latency=d.get("ref_latency"),
                              all_results=d.get("all", []))


class TimeoutException(Exception):
    pass


def run_with_timeout(fn, timeout: float, *args, **kwargs):
    """Run ``fn`` with a wall-clock limit (SIGALRM in the main thread, plain call elsewhere)."""
    if timeout is None or timeout <= 0 or threading.current_thread() is not threading.main_thread():
        return fn(*args, **kwargs)

    def handler(signum, frame):
        raise TimeoutException(f"timed out after {timeout}s")

    old = signal.signal(signal.SIGALRM, handler)
    signal.setitimer(signal.ITIMER_REAL, timeout)
    try:
        return fn(*args, **kwargs)
    finally:
        signal.setitimer(signal.ITIMER_REAL, 0)
        signal.signal(signal.SIGALRM, old)


def _num_workers() -> int:
    n = int(env.TILELANG_AUTO_TUNING_CPU_COUNTS)
    if n <= 0:
        n = max(1, int((os.cpu_count() or 4) * float(env.TILELANG_AUTO_TUNING_CPU_UTILITIES)))
    return max(1, min(n, int(env.TILELANG_AUTO_TUNING_MAX_CPU_COUNT)))


class AutoTuner:

    def __init__(self, fn: Callable, configs: List[dict]):
        self.fn = fn
        self.configs = list(configs)
        self.compile_args = CompileArgs()
        self.profile_args = ProfileArgs()
        self._inputs_cache = None

    @classmethod
    def from_kernel(cls, kernel: Callable, configs: List[dict]):
        return cls(kernel, configs)

    def set_compile_args(self, out_idx=None, target="auto", pass_configs=None, backend=None, **kwargs):
        if backend not in (None, "thread", "process"):
            raise ValueError(f"compile backend must be 'thread' or 'process', got {backend!r}")
        self.compile_args = CompileArgs(out_idx, target, pass_configs, backend)
        return self

    def _prefetch_compile(self, args, kwargs) -> Dict[int, str]:
        """Lower + compile every config in worker processes into the disk kernel cache (see
        ``compile_worker.py``); returns {config index: error} from the workers."""
        import subprocess
        import sys
        import tempfile
        import cloudpickle
        n = min(_num_workers(), len(self.configs))
        errors: Dict[int, str] = {}
        with tempfile.TemporaryDirectory(prefix="tl_tune_compile_") as d:
            procs = []
            env_ = dict(os.environ)
            root = str(Path(__file__).resolve().parents[2])
            paths = [root] + [p_ for p_ in sys.path if p_ and os.path.isdir(p_)]
            env_["PYTHONPATH"] = os.pathsep.join(dict.fromkeys(paths))
            env_["OMP_NUM_THREADS"] = "1"
            for w in range(n):
                share = [(i, c) for i, c in enumerate(self.configs) if i % n == w]
                jp = os.path.join(d, f"job{w}.pkl")
                with open(jp, "wb") as f:
                    cloudpickle.dump(dict(fn=self.fn, args=args, kwargs=kwargs, configs=share), f)
                procs.append((jp, subprocess.Popen([sys.executable, "-m", "tilelang.autotuner.compile_worker", jp],
                                                   env=env_, stdout=subprocess.DEVNULL,
                                                   stderr=subprocess.PIPE, start_new_session=True)))
            for jp, p in procs:
                _, err = p.communicate()
                rp = jp + ".result.json"
                if os.path.exists(rp):
                    with open(rp) as f:
                        errors.update({int(k): v for k, v in json.load(f)["errors"].items()})
                else:
                    logger.warning("autotune compile worker exited with %s: %s", p.returncode,
                                   err.decode(errors="replace")[-300:])
        return errors

    def set_profile_args(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self.profile_args, k, v)
        return self

    # ------------------------------------------------------------------------------
    def _key(self, args, kwargs) -> str:
        from .. import __version__
        fn = getattr(self.fn, "fn", self.fn)
        try:
            src = inspect.getsource(fn)
        except (OSError, TypeError):
            src = fn.__qualname__
        from .capture import get_autotune_inputs
        cap = get_autotune_inputs()
        cap_sig = None if cap is None else [(tuple(getattr(t, "shape", ())), str(getattr(t, "dtype", type(t))))
                                            for t in cap]
        payload = json.dumps({"v": __version__, "src": src, "args": repr(args), "kwargs": repr(sorted(kwargs.items())),
                              "configs": repr(self.configs), "target": str(self.compile_args.target),
                              "captured": repr(cap_sig)}, sort_keys=True)
        return hashlib.sha256(payload.encode()).hexdigest()

    def _bench_isolated(self, args, kwargs, cfg, inputs, warmup, rep, timeout) -> float:
        """Check + time one config in a child process (new session, killed at ``timeout``)."""
        import subprocess
        import sys
        import tempfile
        import cloudpickle
        import torch
        pa = self.profile_args
        with tempfile.TemporaryDirectory(prefix="tl_tune_") as d:
            job = dict(fn=self.fn, args=args, kwargs=kwargs, cfg=cfg, warmup=warmup, rep=rep,
                       supply_type=pa.supply_type, ref_prog=None if pa.skip_check else pa.ref_prog,
                       manual_check_prog=None if pa.skip_check else pa.manual_check_prog, atol=pa.atol, rtol=pa.rtol,
                       max_mismatched_ratio=pa.max_mismatched_ratio)
            with open(os.path.join(d, "job.pkl"), "wb") as f:
                cloudpickle.dump(job, f)
            torch.save([t.detach().cpu() if isinstance(t, torch.Tensor) else t for t in inputs],
                       os.path.join(d, "inputs.pt"))
            env_ = dict(os.environ)
            # the child resolves pickled-by-reference functions exactly as this process does
            root = str(Path(__file__).resolve().parents[2])
            paths = [root] + [p_ for p_ in sys.path if p_ and os.path.isdir(p_)]
            env_["PYTHONPATH"] = os.pathsep.join(dict.fromkeys(paths))
            p = subprocess.Popen([sys.executable, "-m", "tilelang.autotuner.worker", d], env=env_,
                                 start_new_session=True, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
            try:
                _, err = p.communicate(timeout=timeout)
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()
                raise TimeoutException(f"config {cfg} exceeded {timeout}s in its worker process (killed)")
            rp = os.path.join(d, "result.json")
            if not os.path.exists(rp):
                raise RuntimeError(f"worker exited with {p.returncode}: {err.decode(errors='replace')[-500:]}")
            with open(rp) as f:
                res = json.load(f)
        if "latency" not in res:
            raise RuntimeError(res.get("error", "worker failed"))
        return float(res["latency"])

    def _compile(self, args, kwargs, cfg):
        merged = dict(kwargs)
        merged.update(cfg)
        return self.fn(*args, **merged)

    def run(self, *args, warmup=None, rep=None, timeout=None, **kwargs) -> AutotuneResult:
        pa = self.profile_args
        warmup = warmup or pa.warmup
        rep = rep or pa.rep
        timeout = timeout or pa.timeout
        key = self._key(args, kwargs)
        cache_path = Path(env.TILELANG_CACHE_DIR) / "autotuner" / f"{key}.json"
        if env.is_autotune_cache_enabled():
            hit = AutotuneResult.load_from_disk(cache_path)
            if hit is not None and hit.config is not None:
                hit.kernel = self._compile(args, kwargs, hit.config)
                hit.kernel.update_tuner_result(hit.latency, hit.config, hit.ref_latency)
                return hit
        t0 = time.time()
        kernels: List[Any] = [None] * len(self.configs)
        errors: Dict[int, str] = {}
        backend = self.compile_args.backend or os.environ.get("TILELANG_AUTOTUNE_COMPILE", "thread")
        if backend == "process" and env.is_cache_enabled() and len(self.configs) > 1:
            # workers fill the kernel cache; the thread-pool compile below is then all cache hits
            self._prefetch_compile(args, kwargs)
            logger.info("autotune: worker processes compiled %d configs in %.1fs", len(self.configs),
                        time.time() - t0)

        def comp(i):
            try:
                kernels[i] = self._compile(args, kwargs, self.configs[i])
            except Exception as e:  # noqa: BLE001 - invalid configs are skipped
                errors[i] = f"{type(e).__name__}: {e}"

        with ThreadPoolExecutor(_num_workers()) as ex:
            list(ex.map(comp, range(len(self.configs))))
        logger.info("autotune: compiled %d/%d configs in %.1fs", sum(k is not None for k in kernels),
                    len(self.configs), time.time() - t0)
        best = AutotuneResult()
        from .capture import get_autotune_inputs
        captured = get_autotune_inputs()
        inputs = list(captured) if captured is not None else None
        isolate = pa.isolate if pa.isolate is not None else os.environ.get("TILELANG_AUTOTUNE_ISOLATE", "0") == "1"
        for i, k in enumerate(kernels):
            cfg = self.configs[i]
            if k is None:
                best.all_results.append({"config": cfg, "error": errors.get(i)})
                continue
            try:
                prof = k.get_profiler(pa.supply_type)
                if captured is None and (inputs is None or not pa.cache_input_tensors):
                    inputs = pa.supply_prog(k.params) if pa.supply_prog else prof._get_inputs()
                if isolate:
                    lat = self._bench_isolated(args, kwargs, cfg, inputs, warmup, rep, timeout)
                    best.all_results.append({"config": cfg, "latency": lat})
                    if lat < best.latency:
                        best.latency, best.config, best.kernel = lat, cfg, k
                    continue
                if not pa.skip_check:
                    if pa.manual_check_prog is not None:
                        run_with_timeout(pa.manual_check_prog, timeout, k(*inputs), *inputs)
                    elif pa.ref_prog is not None:
                        run_with_timeout(prof.assert_allclose, timeout, pa.ref_prog, inputs, pa.atol, pa.rtol,
                                         pa.max_mismatched_ratio)
                lat = run_with_timeout(prof.do_bench, timeout, None, warmup, rep, input_tensors=inputs)
            except Exception as e:  # noqa: BLE001
                best.all_results.append({"config": cfg, "error": f"{type(e).__name__}: {e}"})
                continue
            best.all_results.append({"config": cfg, "latency": lat})
            if lat < best.latency:
                best.latency, best.config, best.kernel = lat, cfg, k
        if best.kernel is None:
            errs = [r["error"] for r in best.all_results if r.get("error")]
            raise RuntimeError(f"autotune: no config succeeded; errors: {errs[:3]}")
        if pa.ref_prog is not None and inputs is not None:
            try:
                from ..profiler.bench import do_bench
                best.ref_latency = do_bench(lambda: pa.ref_prog(*inputs), warmup=warmup, rep=rep)
            except Exception:  # noqa: BLE001
                best.ref_latency = None
        best.kernel.update_tuner_result(best.latency, best.config, best.ref_latency)
        if env.is_autotune_cache_enabled():
            best.save_to_disk(cache_path)
        return best


class AutoTuneImpl:

    def __init__(self, fn, configs, compile_backend=None, **profile_kwargs):
        self.fn = fn
        self.configs = configs
        self.compile_backend = compile_backend
        self.profile_kwargs = profile_kwargs
        self._cache = {}
        functools.update_wrapper(self, getattr(fn, "fn", fn))

    def __call__(self, *args, **kwargs):
        from ..jit import _freeze
        key = (_freeze(args), _freeze(kwargs))
        if key in self._cache:
            return self._cache[key]
        configs = self.configs(*args, **kwargs) if callable(self.configs) else self.configs
        tuner = AutoTuner(self.fn, configs).set_profile_args(**self.profile_kwargs)
        if self.compile_backend is not None:
            tuner.set_compile_args(backend=self.compile_backend)
        res = tuner.run(*args, **kwargs)
        self._cache[key] = res.kernel
        return res.kernel


def autotune(func: Callable = None, *, configs=None, warmup: int = 25, rep: int = 100, timeout: int = 100,
             supply_type=None, ref_prog=None, supply_prog=None, rtol=1e-2, atol=1e-2, max_mismatched_ratio=0.01,
             skip_check=False, manual_check_prog=None, cache_input_tensors=True, isolate=None,
             compile_backend=None):
    """Decorator: ``@tilelang.autotune(configs=[{...}, ...])`` over ``@tilelang.jit``.
    ``compile_backend="process"``: lower + compile the configs in worker processes."""
    kw = dict(warmup=warmup, rep=rep, timeout=timeout, supply_type=supply_type, ref_prog=ref_prog,
              supply_prog=supply_prog, rtol=rtol, atol=atol, max_mismatched_ratio=max_mismatched_ratio,
              skip_check=skip_check, manual_check_prog=manual_check_prog, cache_input_tensors=cache_input_tensors,
              isolate=isolate)

    def deco(fn):
        return AutoTuneImpl(fn, configs, compile_backend=compile_backend, **kw)

    if func is not None and callable(func):
        return deco(func)
    return deco


from .capture import set_autotune_inputs, get_autotune_inputs, AutotuneInputsCapture  # noqa: E402

__all__ = ["autotune", "AutoTuner", "AutotuneResult", "CompileArgs", "ProfileArgs", "run_with_timeout",
           "set_autotune_inputs", "get_autotune_inputs", "AutotuneInputsCapture"]
