"""Multi-process host logic of the sharded ensemble on CPU
with the gloo backend, world_size 2 and 3.  The device sampler is replaced by
a deterministic stand-in keyed by global member id (the property the HIP
Philox stream has), so these tests check partitioning, the single condition
broadcast and the gather -- not numerics (those are in test_gpu_parity)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ertdiff.ensemble import member_range, sample_ensemble


def test_member_range_partition():
    for n in (0, 1, 7, 64, 1024, 1025):
        for world in (1, 2, 3, 4, 8):
            spans = [member_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


class _Model:
    param_dim = 5


def fake_sampler(model, cond, T, betas, alphas, alpha_bar, P, device, *, num_steps, temperature,
                 mode, noise, seed, member_offset, shared_condition, n_members):
    assert shared_condition and noise == "philox" and cond.shape[0] == 1
    ids = torch.arange(member_offset, member_offset + n_members, dtype=torch.float32)
    # depends on the condition content, the seed and the GLOBAL member id only
    return (cond.sum() + seed + ids[:, None] * 10 + torch.arange(P)[None, :]).float()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _UNetLike:
    """Stand-in with the U-Net's (B, image^2) state shape."""
    image = 4
    param_dim = 16


def _worker(rank, world, port, n_members, q, model_kind="mlp"):
    model = _UNetLike() if model_kind == "unet" else _Model()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = 37
        cond = torch.arange(14 * L, dtype=torch.float32).reshape(14, L) / 100 if rank == 0 else None
        out = sample_ensemble(model, cond, n_members, 10, None, None, None, seed=3, L=L,
                              device=torch.device("cpu"), gather=True, _sampler=fake_sampler)
        # gather=False: no gather collective, each rank returns its own shard
        shard = sample_ensemble(model, cond, n_members, 10, None, None, None, seed=3, L=L,
                                device=torch.device("cpu"), gather=False, _sampler=fake_sampler)
        q.put((rank, out.numpy(), shard.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_members,kind", [(2, 16, "mlp"), (2, 7, "mlp"), (3, 10, "mlp"),
                                                 (2, 1024, "unet")])
def test_sharded_ensemble_gloo(world, n_members, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_members, q, kind))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    L = 37
    cond = torch.arange(14 * L, dtype=torch.float32).reshape(1, 14, L) / 100
    P = (_UNetLike if kind == "unet" else _Model).param_dim
    expect = fake_sampler(_Model(), cond, 10, None, None, None, P, None, num_steps=None,
                          temperature=1.0, mode="hoisted", noise="philox", seed=3,
                          member_offset=0, shared_condition=True, n_members=n_members).numpy()
    shards = []
    for rank, out, shard in sorted(res, key=lambda r: r[0]):
        assert (out == expect).all(), f"rank {rank} gathered ensemble differs from the unsharded one"
        lo, hi = member_range(n_members, world, rank)
        assert shard.shape == (hi - lo, P)
        shards.append(shard)
    # host concatenation of the per-rank shards (the default, collective-free return)
    assert (np.concatenate(shards) == expect).all()


class _TorchBucketOps:
    """allreduce_mean's packing with torch on CPU (the device path uses ertd_concat / ertd_split)."""

    @staticmethod
    def concat(ts):
        return torch.cat([t.reshape(-1) for t in ts])

    @staticmethod
    def split(flat, ts, alpha):
        o = 0
        for t in ts:
            n = t.numel()
            t.copy_((alpha * flat[o:o + n]).view_as(t))
            o += n


def _dp_worker(rank, world, port, q):
    from ertdiff.unet_train import allreduce_mean
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(100 + rank)
        grads = [torch.randn(7, 3, generator=g), torch.randn(5, generator=g), torch.randn(2, 2, 3, 3, generator=g)]
        mine = [t.clone() for t in grads]
        allreduce_mean(grads, dist.group.WORLD, _TorchBucketOps())
        q.put((rank, [t.numpy() for t in mine], [t.numpy() for t in grads]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_dp_gradient_mean_gloo(world):
    """Data-parallel U-Net train step (ertdiff.unet_train.allreduce_mean): every
    rank ends with the mean of all ranks' gradients, tensor shapes intact."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i in range(3):
        want = sum(res[r][0][i] for r in range(world)) / world
        for r in range(world):
            np.testing.assert_allclose(res[r][1][i], want, rtol=1e-6, atol=1e-7)


def fake_conditions_sampler(model, cond, n_samples, T, betas, alphas, alpha_bar, P, device, *,
                            num_steps, temperature, mode, seed, cond_offset, n_conditions_total):
    """Stand-in for ertdiff.sample_conditions: member (r, c) depends on its
    condition's content, the seed and its GLOBAL Philox id r * N + cond_offset + c."""
    nc = cond.shape[0]
    ids = (torch.arange(n_samples)[:, None] * n_conditions_total + cond_offset
           + torch.arange(nc)[None, :]).float()
    csum = cond.reshape(nc, -1).sum(1)[None, :]
    return (csum + seed + ids * 10)[..., None] + torch.arange(P, dtype=torch.float32)


def _cond_worker(rank, world, port, N, q):
    from ertdiff.ensemble import sample_conditions_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = 23
        conds = np.arange(N * 14 * L, dtype=np.float32).reshape(N, 14, L) / 1000  # every rank's host copy
        local, c0, c1 = sample_conditions_sharded(_Model(), conds, 4, 10, None, None, None, seed=5,
                                                  device=torch.device("cpu"),
                                                  _sampler=fake_conditions_sampler)
        q.put((rank, local.numpy(), c0, c1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N", [(2, 509), (2, 3), (3, 8)])
def test_sharded_conditions_gloo(world, N):
    """The test-set evaluation sharded by condition slice (a
    host-side scatter, no collective): each rank's (n_samples, c1 - c0, P)
    block, concatenated along the condition axis, equals the one-process
    (n_samples, N, P) array -- every member keeps its global id r * N + c."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cond_worker, args=(r, world, port, N, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    L = 23
    conds = torch.from_numpy(np.arange(N * 14 * L, dtype=np.float32).reshape(N, 14, L) / 1000)
    expect = fake_conditions_sampler(_Model(), conds, 4, 10, None, None, None, _Model.param_dim, None,
                                     num_steps=None, temperature=1.0, mode="hoisted", seed=5,
                                     cond_offset=0, n_conditions_total=N).numpy()
    spans = [(c0, c1) for _, _, c0, c1 in res]
    assert spans == [member_range(N, world, r) for r in range(world)]
    got = np.concatenate([local for _, local, _, _ in res], axis=1)
    assert got.shape == (4, N, _Model.param_dim)
    assert (got == expect).all()
