"""Developer tools: static roofline analysis and layout rendering (reference ``tilelang/tools``)."""
from .Analyzer import Analyzer, AnalysisResult, ARCH_CONFIGS  # noqa: F401
from .plot_layout import plot_layout, layout_text, layout_svg  # noqa: F401
