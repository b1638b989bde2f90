"""Compiler passes (reference ``tilelang/transform/__init__.py``)."""
from .pass_config import PassConfigKey  # noqa: F401
from .layout_inference import infer_layouts, LayoutInference, LayoutConflictError  # noqa: F401
from .pipeline import inject_software_pipeline  # noqa: F401
from .lower_tile_op import lower_tile_ops, LoweringError  # noqa: F401
from .thread_sync import insert_thread_sync  # noqa: F401
from .lds_plan import plan_lds  # noqa: F401
