"""Full-batch L-BFGS with a strong-Wolfe line search, the solver behind
MultilayerPerceptronClassifier(solver='l-bfgs') (mllib_multilayer_perceptron_classifier.py:32-35).

Spark's MLP trains with Breeze ``LBFGS(maxIter, m=10, tolerance)`` on the block-averaged loss
(SURVEY.md App. A.1).  This is a device-resident re-implementation: the parameter vector, the
correction pairs and the two-loop recursion live on the tensor's device; the objective closure
evaluates the fused full-batch loss+gradient (sparkmi/ops/mlp.py) — on an executor group it
is already all-reduced over executors, replacing Spark's treeAggregate.
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


def strong_wolfe(fg, x, d, f0, g0, t=1.0, c1=1e-4, c2=0.9, max_iter=10):
    """Returns (t, f_new, g_new, n_evals)."""
    gtd0 = float(g0 @ d)
    t_prev, f_prev, gtd_prev = 0.0, f0, gtd0
    g_prev = g0
    evals = 0
    f_new, g_new = None, None
    bracket = None
    for i in range(max_iter):
        f_new, g_new = fg(x + t * d)
        evals += 1
        gtd_new = float(g_new @ d)
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
        f_new, g_new = fg(x + t * d)
        evals += 1
        gtd_new = float(g_new @ d)
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


class LBFGS:
    def __init__(self, max_iter=100, m=10, tol=1e-6):
        self.max_iter, self.m, self.tol = max_iter, m, tol
        self.objective_history = []
        self.iterations = 0
        self.evaluations = 0

    def minimize(self, fg, x0: torch.Tensor):
        """fg(x) -> (float loss, grad tensor).  Returns the optimum (same device/dtype as x0)."""
        x = x0.clone()
        f, g = fg(x)
        self.evaluations = 1
        self.objective_history = [float(f)]
        S, Y, rho = [], [], []
        for it in range(self.max_iter):
            if float(g.norm()) <= 1e-12:
                break
            q = g.clone()
            alphas = []
            for s, y, r in zip(reversed(S), reversed(Y), reversed(rho)):
                a = r * float(s @ q)
                alphas.append(a)
                q.add_(y, alpha=-a)
            if S:
                gamma = float(S[-1] @ Y[-1]) / float(Y[-1] @ Y[-1])
                q.mul_(gamma)
            for (s, y, r), a in zip(zip(S, Y, rho), reversed(alphas)):
                b = r * float(y @ q)
                q.add_(s, alpha=a - b)
            d = -q
            if float(g @ d) >= 0:  # not a descent direction: reset memory
                S, Y, rho = [], [], []
                d = -g
            t0 = 1.0 if S else min(1.0, 1.0 / max(float(g.abs().sum()), 1e-12))
            t, f_new, g_new, ev = strong_wolfe(fg, x, d, float(f), g, t=t0)
            self.evaluations += ev
            s = t * d
            x = x + s
            y = g_new - g
            sy = float(s @ y)
            if sy > 1e-10:
                S.append(s)
                Y.append(y)
                rho.append(1.0 / sy)
                if len(S) > self.m:
                    S.pop(0), Y.pop(0), rho.pop(0)
            f_old = float(f)
            f, g = float(f_new), g_new
            self.objective_history.append(f)
            self.iterations = it + 1
            denom = max(abs(f), abs(f_old), 1e-8)
            if abs(f_old - f) / denom < self.tol:
                break
        return x
