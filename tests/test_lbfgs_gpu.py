"""Device L-BFGS (csrc/kernels/lbfgs.hip) and the GPU MLlib fit (sparkmi/ml/classification.py).

* the two-loop recursion kernel and the pair-update kernel against the float64 torch
  implementation of the same ring-buffer algorithm (random pairs, a full ring that wrapped, a
  rejected pair, reset);
* a GPU fit of the MLlib MLP (fused HIP objective + device L-BFGS) learns, and its objective
  trajectory follows the float64 CPU fit;
* a 2-executor GPU fit (two processes sharing the device, gloo) is bit-identical to the
  1-executor GPU fit (slab-ordered reduction + deterministic MLP kernel).
"""
import numpy as np
import pytest
import torch

from sparkmi.optim.lbfgs import _Memory

pytestmark = pytest.mark.gpu
dev = torch.device("cuda")


def _pairs(mem, n, k, g):
    for _ in range(k):
        d = torch.randn(n, generator=g, dtype=torch.float64)
        g_old = torch.randn(n, generator=g, dtype=torch.float64)
        g_new = g_old + 0.5 * d + 0.1 * torch.randn(n, generator=g, dtype=torch.float64)
        yield d, g_new, g_old


def test_two_loop_and_update_kernels_match_torch():
    n, m = 3000, 5
    g = torch.Generator().manual_seed(0)
    xc = torch.zeros(n, dtype=torch.float64)
    xg = torch.zeros(n, dtype=torch.float32, device=dev)
    mc, mg = _Memory(m, xc), _Memory(m, xg)
    assert mg.native and not mc.native
    for i, (d, gn, go) in enumerate(_pairs(None, n, 8, g)):  # 8 > m: the ring wraps
        if i == 6:
            gn = go - d  # s.y < 0: rejected by both
        t = 0.7
        mc.update(xc, d, t, gn, go)
        mg.update(xg, d.float().to(dev), t, gn.float().to(dev), go.float().to(dev))
        q = torch.randn(n, generator=g, dtype=torch.float64)
        dc, dg = torch.empty_like(q), torch.empty(n, device=dev)
        rc = mc.direction(q, dc)
        rg = mg.direction(q.float().to(dev), dg)
        assert rg[3] == rc[3] == min(i + 1 - (i >= 6), m), (rg[3], rc[3], i)
        torch.testing.assert_close(dg.cpu().double(), dc, atol=1e-4, rtol=1e-4)
        for a, b in zip(rg[:3], rc[:3]):
            assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), (rg, rc)
    torch.testing.assert_close(xg.cpu().double(), xc, atol=1e-5, rtol=1e-5)
    # reset: steepest descent, memory dropped
    q = torch.randn(n, generator=g, dtype=torch.float64)
    dg = torch.empty(n, device=dev)
    r = mg.direction(q.float().to(dev), dg, True)
    torch.testing.assert_close(dg.cpu().double(), -q, atol=1e-6, rtol=1e-6)
    assert r[3] == 0 and int(mg.st[1]) == 0


def _iris():
    from sparkmi.api import Session
    from sparkmi.data.synthetic import iris_libsvm_text
    s = Session.builder.appName("lbfgs_gpu").config("spark.executor.instances", "1").getOrCreate()
    df = s.read.libsvm(iris_libsvm_text(150, seed=3), text=True)
    return s, df


def test_gpu_fit_learns_and_tracks_cpu():
    from sparkmi.ml import MulticlassClassificationEvaluator, MultilayerPerceptronClassifier
    s, df = _iris()
    try:
        train, test = df.randomSplit([0.6, 0.4], 1234)
        kw = dict(maxIter=30, layers=[4, 5, 4, 3], blockSize=30, seed=1234, numExecutors=1)
        mg = MultilayerPerceptronClassifier(device="cuda", **kw).fit(train)
        mc = MultilayerPerceptronClassifier(device="cpu", **kw).fit(train)
        hg, hc = mg.summary.objectiveHistory, mc.summary.objectiveHistory
        assert hg[-1] < 0.5 * hg[0]
        for a, b in list(zip(hg, hc))[:10]:  # fp32 device vs fp64 host: same early trajectory
            assert abs(a - b) <= 1e-3 * abs(b) + 1e-5, (a, b)
        acc = MulticlassClassificationEvaluator(metricName="accuracy").evaluate(mg.transform(test))
        assert acc > 0.8, acc
    finally:
        s.stop()


def test_gpu_two_executor_fit_bit_identical():
    from sparkmi.ml import MultilayerPerceptronClassifier
    s, df = _iris()
    try:
        kw = dict(maxIter=25, layers=[4, 5, 4, 3], blockSize=30, seed=7, device="cuda")
        m1 = MultilayerPerceptronClassifier(numExecutors=1, **kw).fit(df)
        m2 = MultilayerPerceptronClassifier(numExecutors=2, **kw).fit(df)
        assert m2._num_executors == 2
        np.testing.assert_array_equal(m2.weights.toArray(), m1.weights.toArray())
    finally:
        s.stop()
