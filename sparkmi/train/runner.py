"""Training-step executor: eager or HIP-graph-captured, optionally data-parallel.

A "step" = dropout-seed bump -> forward -> loss -> backward (gradients land in the flat fp32
buffer) -> gradient all-reduce (data-parallel) -> fused optimizer launch.
With ``graph=True`` the step's kernels are captured once into a hipGraph after a few eager
warm-up steps and then replayed: one host launch per step instead of hundreds, which matters
at the reference's small per-GPU batches.  Inputs are copied into static
device buffers before each replay.
  * one executor: the whole step (optimizer included) is one graph;
  * data-parallel: the graph holds forward + backward; the gradient buckets are then
    all-reduced by RCCL (a few large collectives over the flat buffer) and the optimizer runs
    as one launch.  Collectives stay outside the graph, so no RCCL-in-capture dependency;
    eager data-parallel steps instead overlap the bucket all-reduces with backward.
  * data-parallel with ``split_fn`` (a loss whose autograd graph is cut in two, e.g.
    Transformer.training_step_split at the encoder output): the step is TWO graphs — G1 =
    forward + backward of the upper segment (decoder + vocab projection), G2 = backward of the
    lower segment (encoder).  Buckets whose parameters all became final inside G1 are
    all-reduced on RCCL's stream while G2 replays, so most of the gradient traffic hides under
    the encoder backward; the rest is reduced after G2.  Still no collective inside a graph.
"""
import torch

from ..ops import _grad


class StepRunner:
    def __init__(self, model, loss_fn, optimizer, ddp=None, graph=False, warmup_eager=3, split_fn=None):
        self.model = model
        self.loss_fn = loss_fn          # loss_fn(model, *batch) -> scalar loss tensor
        self.split_fn = split_fn        # split_fn(model, *batch) -> (loss, leaf, root), see module doc
        self.graph2 = None
        self.early_buckets = []
        self._split_keep = None
        self.opt = optimizer
        self.ddp = ddp
        self.graph_requested = graph
        self.warmup_eager = warmup_eager
        self.graph = None
        self.static_in = None
        self.static_loss = None
        self.steps = 0
        if ddp is not None:
            optimizer.grad_scale = ddp.grad_scale

    @property
    def _dp(self):
        return self.ddp is not None and self.ddp.world > 1

    def _fwd_bwd(self, *batch):
        rng = getattr(self.model, "rng", None)
        if rng is not None:
            rng.advance()
        loss = self.loss_fn(self.model, *batch)
        loss.backward()
        _grad.join()
        return loss.detach()

    def _eager(self, *batch):
        loss = self._fwd_bwd(*batch)
        if self.ddp is not None:
            self.ddp.finish()
        self.opt.step()
        return loss

    def _fwd_bwd_split(self, *batch):
        rng = getattr(self.model, "rng", None)
        if rng is not None:
            rng.advance()
        loss, leaf, root = self.split_fn(self.model, *batch)
        loss.backward()
        _grad.join()
        return loss.detach(), leaf, root

    def _capture_split(self):
        """G1 = forward + upper backward, G2 = lower backward (shares G1's memory pool); records
        which gradient buckets are final after G1."""
        ready = set()
        listener = _grad.add_listener(lambda p: ready.add(id(p)))
        g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g1):
                self.static_loss, leaf, root = self._fwd_bwd_split(*self.static_in)
        finally:
            _grad.remove_listener(listener)
        late = set()
        listener = _grad.add_listener(lambda p: late.add(id(p)))
        try:
            with torch.cuda.graph(g2, pool=g1.pool()):
                root.backward(leaf.grad)
                _grad.join()
        finally:
            _grad.remove_listener(listener)
        ready -= late  # a gradient also accumulated in the lower segment is not final after G1
        self._split_keep = (leaf, root)  # G2 reads leaf.grad / root's saved tensors at fixed addresses
        self.graph, self.graph2 = g1, g2
        self.ddp.align_buckets(ready)
        self.early_buckets = self.ddp.complete_buckets(ready)

    def _capture(self, batch):
        """Record one step into a HIP graph.  Capture only records (nothing executes), so no
        extra optimizer updates happen here: the ``warmup_eager`` eager steps before it already
        did every lazy initialisation (allocator pools, GEMM autotuning, library handles), and
        the caller replays the graph for the current step right after."""
        self.static_in = [b.clone() for b in batch]
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        if self._dp and self.split_fn is not None:
            self.ddp.set_overlap(False)
            self._capture_split()
            return
        if self._dp:
            self.ddp.set_overlap(False)  # no collective may be enqueued during capture
            with torch.cuda.graph(g):
                self.static_loss = self._fwd_bwd(*self.static_in)
        else:
            with torch.cuda.graph(g):
                self.static_loss = self._eager(*self.static_in)
        self.graph = g

    def step(self, *batch):
        self.steps += 1
        use_graph = self.graph_requested and batch[0].is_cuda
        if not use_graph or self.steps <= self.warmup_eager:
            return self._eager(*batch)
        if self.graph is None:
            self._capture(batch)  # then replayed below for this step
        for dst, src in zip(self.static_in, batch):
            dst.copy_(src, non_blocking=True)
        self.graph.replay()
        if self.graph2 is not None:
            for b in self.early_buckets:   # decoder buckets: RCCL runs under the encoder backward
                self.ddp.launch(b)
            self.graph2.replay()
        if self._dp:
            self.ddp.finish()   # bucketed RCCL all-reduce of the flat gradient buffer
            self.opt.step()
        return self.static_loss
