"""Full-batch L-BFGS with a strong-Wolfe line search, the solver behind
MultilayerPerceptronClassifier(solver='l-bfgs') (mllib_multilayer_perceptron_classifier.py:32-35).

Spark's MLP trains with Breeze ``LBFGS(maxIter, m=10, tolerance)`` on the block-averaged loss
(SURVEY.md App. A.1), the driver running the recursion over treeAggregate'd gradients.  Here
everything is device-resident: the parameter vector, the correction pairs (S, Y ring buffers),
rho and the ring state live on the tensor's device, and on an MI355X the two-loop recursion and
the pair update are single HIP launches (csrc/kernels/lbfgs.hip) — only the line-search scalars
(f, g.d, |g|) reach the host.  The objective closure evaluates the fused loss+gradient
(sparkmi/ops/mlp.py); on an executor group it all-reduces them over the executors
(sparkmi/ml/classification.py: _fit_executor), replacing Spark's treeAggregate, and every
executor runs the same deterministic recursion on the reduced values.  CPU tensors use the same
algorithm in torch (float64 when the caller works in float64).
Convergence (Breeze FirstOrderMinimizer semantics): stop when the relative improvement of the
objective over the last iteration, |f_k - f_{k-1}| / max(|f_k|, |f_{k-1}|, 1e-8), falls below
``tol``, when the gradient norm is ~0, or after ``max_iter`` iterations.
"""
import torch


def _cubic_min(x1, f1, g1, x2, f2, g2, lo, hi):
    d1 = g1 + g2 - 3 * (f1 - f2) / (x1 - x2)
    d2sq = d1 * d1 - g1 * g2
    if d2sq >= 0:
        d2 = d2sq ** 0.5
        if x1 <= x2:
            t = x2 - (x2 - x1) * ((g2 + d2 - d1) / (g2 - g1 + 2 * d2))
        else:
            t = x1 - (x1 - x2) * ((g1 + d2 - d1) / (g1 - g2 + 2 * d2))
        return min(max(t, lo), hi)
    return (lo + hi) / 2


def strong_wolfe(ev, x, d, f0, g0, gtd0, t=1.0, c1=1e-4, c2=0.9, max_iter=10):
    """ev(x_t) -> (f, g, g.d) with host floats f, g.d.  Returns (t, f_new, g_new, n_evals)."""
    t_prev, f_prev, gtd_prev = 0.0, f0, gtd0
    g_prev = g0
    evals = 0
    f_new, g_new = None, None
    bracket = None
    for i in range(max_iter):
        f_new, g_new, gtd_new = ev(torch.add(x, d, alpha=t))
        evals += 1
        if f_new > f0 + c1 * t * gtd0 or (i > 0 and f_new >= f_prev):
            bracket = [(t_prev, f_prev, gtd_prev, g_prev), (t, f_new, gtd_new, g_new)]
            break
        if abs(gtd_new) <= -c2 * gtd0:
            return t, f_new, g_new, evals
        if gtd_new >= 0:
            bracket = [(t, f_new, gtd_new, g_new), (t_prev, f_prev, gtd_prev, g_prev)]
            break
        t_next = _cubic_min(t_prev, f_prev, gtd_prev, t, f_new, gtd_new, t + 0.01 * (t - t_prev), t * 10)
        t_prev, f_prev, gtd_prev, g_prev = t, f_new, gtd_new, g_new
        t = t_next
    if bracket is None:
        return t, f_new, g_new, evals
    # zoom
    for _ in range(max_iter):
        (tl, fl, gl, gvl), (th, fh, gh, gvh) = bracket
        lo, hi = min(tl, th), max(tl, th)
        if hi - lo < 1e-12:
            break
        t = _cubic_min(tl, fl, gl, th, fh, gh, lo + 0.1 * (hi - lo), hi - 0.1 * (hi - lo))
        f_new, g_new, gtd_new = ev(torch.add(x, d, alpha=t))
        evals += 1
        if f_new > f0 + c1 * t * gtd0 or f_new >= fl:
            bracket[1] = (t, f_new, gtd_new, g_new)
        else:
            if abs(gtd_new) <= -c2 * gtd0:
                return t, f_new, g_new, evals
            if gtd_new * (th - tl) >= 0:
                bracket[1] = bracket[0]
            bracket[0] = (t, f_new, gtd_new, g_new)
    tl, fl, _, gvl = bracket[0]
    return tl, fl, gvl, evals


class _Memory:
    """Correction pairs on x's device: S, Y [m, n], rho [m], st = {head, count} (int32)."""

    def __init__(self, m, x):
        n = x.numel()
        self.m, self.n = m, n
        self.S = torch.zeros(m, n, dtype=x.dtype, device=x.device)
        self.Y = torch.zeros(m, n, dtype=x.dtype, device=x.device)
        self.rho = torch.zeros(m, dtype=x.dtype, device=x.device)
        self.st = torch.zeros(2, dtype=torch.int32, device=x.device)
        self.out = torch.zeros(4, dtype=torch.float32, device=x.device)
        self.native = x.is_cuda and x.dtype == torch.float32
        if self.native:
            from .. import _native
            self._C, self._stream = _native.C(), _native.stream
        else:
            self.head, self.count = 0, 0

    def direction(self, g, d, reset=False):
        """d = -H g; returns (g.d, |g|_1, |g|_2^2, pairs used) as host values (one read)."""
        if self.native:
            self._C.lbfgs_direction(self.S.data_ptr(), self.Y.data_ptr(), self.rho.data_ptr(), self.st.data_ptr(),
                                    self.m, self.n, g.data_ptr(), d.data_ptr(), self.out.data_ptr(), int(reset),
                                    self._stream())
            gd, g1, g2, cnt = self.out.tolist()
            return gd, g1, g2, int(cnt)
        if reset:
            self.count = 0
        q = g.clone()
        alphas = []
        for j in range(self.count):
            k = (self.head - 1 - j) % self.m
            a = self.rho[k] * (self.S[k] @ q)
            alphas.append(a)
            q -= a * self.Y[k]
        if self.count:
            k = (self.head - 1) % self.m
            yy = self.Y[k] @ self.Y[k]
            q *= (1.0 / self.rho[k]) / (yy if float(yy) > 0 else 1.0)
        for j in range(self.count - 1, -1, -1):
            k = (self.head - 1 - j) % self.m
            b = self.rho[k] * (self.Y[k] @ q)
            q += (alphas[j] - b) * self.S[k]
        d.copy_(-q)
        return float(g @ d), float(g.abs().sum()), float(g @ g), self.count

    def update(self, x, d, t, g_new, g_old, eps=1e-10):
        """x += t d; store (t d, g_new - g_old) when it satisfies the curvature condition."""
        if self.native:
            self._C.lbfgs_update(self.S.data_ptr(), self.Y.data_ptr(), self.rho.data_ptr(), self.st.data_ptr(),
                                 self.m, self.n, d.data_ptr(), float(t), g_new.data_ptr(), g_old.data_ptr(),
                                 x.data_ptr(), float(eps), self._stream())
            return
        s = t * d
        y = g_new - g_old
        sy = float(s @ y)
        if sy > eps:
            self.S[self.head].copy_(s)
            self.Y[self.head].copy_(y)
            self.rho[self.head] = 1.0 / sy
            self.head = (self.head + 1) % self.m
            self.count = min(self.count + 1, self.m)
        x.add_(s)


class LBFGS:
    def __init__(self, max_iter=100, m=10, tol=1e-6):
        self.max_iter, self.m, self.tol = max_iter, m, tol
        self.objective_history = []
        self.iterations = 0
        self.evaluations = 0

    def minimize(self, fg, x0: torch.Tensor):
        """fg(x) -> (loss: float or 0-d tensor, grad: NEW tensor shaped like x).  Returns the
        optimum (same device/dtype as x0)."""
        x = x0.detach().clone().contiguous()
        mem = _Memory(self.m, x)
        d = torch.empty_like(x)

        def ev(xt):
            f, g = fg(xt)
            if torch.is_tensor(f):
                f, gd = torch.stack([f.detach().reshape(()).to(g.dtype), (g * d).sum()]).tolist()
            else:
                gd = float((g * d).sum())
            return float(f), g.contiguous(), gd

        f, g = fg(x)
        f = float(f)
        g = g.contiguous()
        self.evaluations = 1
        self.objective_history = [f]
        for it in range(self.max_iter):
            gtd, g1, g2, pairs = mem.direction(g, d)
            if g2 <= 1e-24:
                break
            if gtd >= 0:  # not a descent direction: drop the memory, steepest descent
                gtd, g1, g2, pairs = mem.direction(g, d, True)
            t0 = min(1.0, 1.0 / max(g1, 1e-12)) if pairs == 0 else 1.0
            t, f_new, g_new, n_ev = strong_wolfe(ev, x, d, f, g, gtd, t=t0)
            self.evaluations += n_ev
            mem.update(x, d, t, g_new, g)
            f_old = f
            f, g = f_new, g_new
            self.objective_history.append(f)
            self.iterations = it + 1
            if abs(f_old - f) / max(abs(f), abs(f_old), 1e-8) < self.tol:
                break
        return x
