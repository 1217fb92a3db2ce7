"""Multi-GPU layouts of the fast-GP path.

* Independent GPs (config C4, random shifts): replicas only -- each rank owns its own GPs, no
  collective on the data path (bench.py: shard_seeds / max_over_ranks).
* One GP with many outputs sharing its hyper-parameters (config C5: FastGPLattice, shape_batch=[B],
  default shape_scale=[1] / shape_lengthscales=[d]): the outputs are split across the ranks.  The MLL
  (fastgps/abstract_gp.py:252-261, util.py:364-370) depends on the data only through
  Y_k = sum_b |ytilde_bk|^2, so each rank transforms its own outputs, forms its partial Y, and ONE
  all-reduce (SUM, n float64) makes Y global; every rank then runs the identical device-resident fit
  (same inputs, same kernels -> same parameters on every rank, no per-iteration exchange).  coeffs /
  post_mean / post_var of each output stay on the rank that owns it.

The only collective is `allreduce_sum_` (RCCL over xGMI with the "nccl" backend, gloo on CPU).
"""
import numpy as np
import torch


def output_shard(total, rank, world):
    """Contiguous [start, stop) range of the outputs owned by `rank` (sizes differ by at most one)."""
    assert 0 <= rank < world and total >= world, "need at least one output per rank"
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def allreduce_sum_(t, group=None):
    """In-place SUM all-reduce over the process group (identity without an initialised group)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if t.is_cuda and dist.get_backend(group) == "gloo":
            # gloo reduces host memory: stage the device tensor (RCCL / "nccl" reduces it in place)
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def fit_sharded(gp, total_outputs, group=None, iterations=5000, lr=None, stop_crit_improvement_threshold=5e-2,
                stop_crit_wait_iterations=10, store_hists=False, store_loss_hist=False, verbose=0, verbose_indent=4):
    """MLL fit of a multi-output GP whose outputs are sharded over the ranks of `group`.

    `gp` holds this rank's outputs (shape_batch = [local outputs]) and hyper-parameters shared by all
    outputs; `total_outputs` is the global output count.  Returns what `gp.fit(...)` returns on the
    unsharded GP (the loss uses d_out = total_outputs, fastgps/abstract_gp.py:235,256)."""
    assert gp._fused_ok(), "fit_sharded needs the fused MLL path (default transforms, single task)"
    pb, G = gp._problem_batch()
    assert G == 1, "fit_sharded: hyper-parameters must be shared by all outputs (per-output ones shard as replicas)"
    assert isinstance(iterations, int) and iterations >= 0
    ysq = gp._ysq(pb, G).contiguous()
    allreduce_sum_(ysq, group)
    hists = dict(loss=store_hists or store_loss_hist,
                 scale=store_hists, lengthscales=store_hists, noise=store_hists, task_kernel=store_hists)
    stop = (np.log(1 + stop_crit_improvement_threshold), stop_crit_wait_iterations)
    return gp._fit_fused(iterations, 1e-1 if lr is None else lr, stop, hists, verbose, verbose_indent, ysq=ysq,
                         d_out=int(total_outputs))
