"""HIP-graph capture of a whole training step (forward + backward + gradient
all-reduce + fused optimizer update).

MI355X-first replacement for a tracing compiler: the step's ~600 kernel
launches are recorded once into a hipGraph and replayed with a single
``hipGraphLaunch``, removing per-kernel host launch cost (~3-4 us each on
ROCm 7.2, MI355X_MICROARCH "graph-replay-floor").  Requirements met by the
rest of the framework:

* static inputs (the caller owns fixed ``x``/``y`` buffers and refills them);
* the optimizer's hyper-parameters are read from device memory, refreshed by
  :meth:`FusedOptimizer.prepare_step` BEFORE each replay (outside the graph);
* gradients live in the flat arena (fixed addresses), zeroed inside the graph.
"""
from __future__ import annotations

import torch


class GraphedStep:
    def __init__(self, fwd_bwd, opt, reducer=None, warmup=3):
        self.fwd_bwd, self.opt, self.reducer = fwd_bwd, opt, reducer
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._eager_body()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        self.opt.prepare_step()
        with torch.cuda.graph(self.graph):
            self.out = self._body()
        torch.cuda.synchronize()

    def _eager_body(self):
        self.opt.zero_grad()
        out = self.fwd_bwd()
        if self.reducer is not None:
            self.reducer.finish()
        self.opt.step()
        return out

    def _body(self):
        self.opt.zero_grad()
        out = self.fwd_bwd()
        if self.reducer is not None:
            self.reducer.finish()
        self.opt.step_kernels()
        return out

    def __call__(self):
        self.opt.iterations += 1
        self.opt.prepare_step()
        self.graph.replay()
        return self.out


def capture_train_step(fwd_bwd, opt, reducer=None, warmup=3):
    return GraphedStep(fwd_bwd, opt, reducer, warmup)
