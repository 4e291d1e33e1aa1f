"""Host logic of tools/fullscale.py (CPU): the report a failed factorisation carries
(``lead_report``: the saved leading block's host Cholesky and its entries against a fresh
build), and the synthetic image generator the full-scale legs and their GPU tests share."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tools"))

import fullscale  # noqa: E402


def _model(X):
    """a PD Gram stand-in for model(X): X Xᵀ + I"""
    F = X.reshape(len(X), -1).double()
    return F @ F.T + torch.eye(len(X), dtype=torch.float64)


def test_lead_report_clean_block():
    X = fullscale.mnist_like(24, 1, 28, 0)
    rep = fullscale.lead_report(_model, X, _model(X[:16]))
    assert "host Cholesky of the saved block ok" in rep
    assert "0 entries differ" in rep


def test_lead_report_names_a_corrupted_entry():
    X = fullscale.mnist_like(24, 1, 28, 0)
    lead = _model(X[:16]).clone()
    lead[3, 5] = lead[5, 3] = 1e6                 # breaks PD and differs from a fresh build
    lead[7, 9] = float("nan")
    rep = fullscale.lead_report(_model, X, lead)
    assert "host Cholesky of the saved block fails" in rep
    assert "2 entries differ" in rep              # the upper triangle only: (3, 5), (7, 9)
    assert "(3, 5, 1000000.0" in rep and "(7, 9, nan" in rep


def test_mnist_like_images():
    x = fullscale.mnist_like(64, 3, 32, 0)
    assert x.shape == (64, 3, 32, 32) and x.dtype == torch.float64
    assert torch.equal(x, fullscale.mnist_like(64, 3, 32, 0))
    v = x.numpy()
    assert np.all(v[..., :4, :] == 0) and np.all(v[..., -4:, :] == 0)
    assert np.all(v[..., :4] == 0) and np.all(v[..., -4:] == 0)
    assert np.array_equal(np.round(v * 255), v * 255) and v.max() <= 1.0
    inner = v[..., 4:-4, 4:-4]
    assert 0.55 < (inner == 0).mean() < 0.66         # ~60% zero pixels (+ the k = 0 draws)
