"""Model explanation: TreeSHAP explainer API and SHAP plots."""
from .shap import Explanation, TreeExplainer, bar_plot, force_data, summary_plot

__all__ = ["TreeExplainer", "Explanation", "bar_plot", "summary_plot", "force_data"]
