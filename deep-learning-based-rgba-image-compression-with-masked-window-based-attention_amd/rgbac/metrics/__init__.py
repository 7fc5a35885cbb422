"""Evaluation metrics (reference: metrics/), computed by HIP kernels."""
