"""CPU: pins the oracle's gradient and update beyond the reference's two known-answer tests.

The reference's tests pin the forward (FactorizationMachinesSuite.scala:24-75) and VectorSum
(:77-102) only; its gradient, update and L1 have no fixture.  Here they are pinned
by a second, independent derivation: torch's fp64 automatic differentiation of the FM forward
(whose oracle form IS pinned by the KAT, test_oracle.py).

  * deltaVi (Model.scala:201-204) = d yhat / d v_i for every entry -- per entry, by autograd;
  * the V-update of one step (SGD.scala:146, 151-154, 172-181): the sum of g_V = deltaVi (yhat - y)
    over a feature's entries is the gradient of 1/2 sum_s (yhat_s - y_s)^2 wrt V, so
    V' = S_lambda(V - (eta / m) * dL/dV) on touched rows and S_lambda(V) on the other present rows;
  * deltaWi = x = d yhat / d w_i (Model.scala:200).  The w-update itself keeps the reference's
    precedence bug g_w = x * yhat - y (SGD.scala:145), which is no derivative of
    anything: it stays pinned by the reference expression alone and is recomputed here from it.
"""

import math

import numpy as np
import pytest
import torch

from oracle import fm_ref as R
from problems import make_problem


def _torch_forward(w, V, csr):
    rows = torch.from_numpy(np.repeat(np.arange(csr.n_rows), np.diff(csr.row_ptr)))
    ids = torch.from_numpy(csr.col.astype(np.int64))
    x = torch.from_numpy(csr.val)
    Vx = V[ids] * x[:, None]
    S = torch.zeros(csr.n_rows, V.shape[1], dtype=torch.float64).index_add(0, rows, Vx)
    vv = torch.zeros(csr.n_rows, dtype=torch.float64).index_add(0, rows, (Vx * Vx).sum(1))
    wx = torch.zeros(csr.n_rows, dtype=torch.float64).index_add(0, rows, w[ids] * x)
    return 0.5 * ((S * S).sum(1) - vv) + wx


@pytest.mark.parametrize("seed,k", [(1, 4), (2, 7)])
def test_delta_vi_is_the_derivative_of_the_forward(seed, k):
    F = 40
    csr, ids, w, V = make_problem(seed, 30, F, k, 6, zero_frac=0.1)
    model = R.Model.empty(F, k)
    model.load(ids, w, V)
    pred, _, dw, dv = R.loss_grad(model, csr)
    wt = torch.tensor(w, requires_grad=True)
    Vt = torch.tensor(V, requires_grad=True)
    yhat = _torch_forward(wt, Vt, csr)
    rows = np.repeat(np.arange(csr.n_rows), np.diff(csr.row_ptr))
    np.testing.assert_allclose(pred, yhat.detach().numpy()[rows], rtol=1e-12, atol=1e-12)
    for s in range(csr.n_rows):
        e0, e1 = csr.row_ptr[s], csr.row_ptr[s + 1]
        if e0 == e1:
            continue
        gw, gV = torch.autograd.grad(yhat[s], (wt, Vt), retain_graph=True)
        for e in range(e0, e1):
            i = int(csr.col[e])
            np.testing.assert_allclose(dv[e], gV[i].numpy(), rtol=1e-12, atol=1e-14)
            assert dw[e] == pytest.approx(float(gw[i]), rel=1e-12, abs=1e-14)


@pytest.mark.parametrize("seed,k,reg", [(3, 4, 1e-4), (4, 8, 0.0), (5, 3, 2e-2)])
def test_step_v_update_is_the_autograd_gradient_step(seed, k, reg):
    F, t, step = 60, 3, 0.4
    csr, ids, w, V = make_problem(seed, 50, F, k, 7, hot=5)
    present = np.ones(F, bool)
    present[::7] = False  # some rows absent; the batch may still touch them
    model = R.Model.empty(F, k)
    model.load(ids[present], w[present], V[present])
    w0, V0 = model.w.copy(), model.V.copy()
    R.sgd_step_fast(model, csr, t, step, reg)
    eta = step / math.sqrt(t)
    lam = eta * reg
    m = csr.n_rows
    Vt = torch.tensor(V0, requires_grad=True)
    yhat = _torch_forward(torch.tensor(w0), Vt, csr)
    has = torch.from_numpy(np.diff(csr.row_ptr) > 0)
    y = torch.from_numpy(csr.label)
    L = 0.5 * ((yhat - y)[has] ** 2).sum()
    (gV,) = torch.autograd.grad(L, Vt)
    touched = np.unique(csr.col)
    rows = present.copy()
    rows[touched] = True
    Vexp = V0.copy()
    Vexp[touched] = V0[touched] - (eta / m) * gV.numpy()[touched]
    Vexp[rows] = R.soft_threshold(Vexp[rows], lam)
    np.testing.assert_allclose(model.V, Vexp, rtol=1e-12, atol=1e-15)
    # w: the reference expression g_w = x * yhat - y (P1), recomputed outside the oracle
    yh = yhat.detach().numpy()
    srow = np.repeat(np.arange(m), np.diff(csr.row_ptr))
    gw = np.zeros(F)
    np.add.at(gw, csr.col, csr.val * yh[srow] - csr.label[srow])
    wexp = w0.copy()
    wexp[touched] = w0[touched] - (gw[touched] / m) * eta
    wexp[rows] = R.soft_threshold(wexp[rows], lam)
    np.testing.assert_allclose(model.w, wexp, rtol=1e-12, atol=1e-15)
    assert np.array_equal(model.present, rows)
