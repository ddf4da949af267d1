"""Data-parallel exchange (lcclip/dp.py) on CPU with the gloo backend, world sizes 2 and 4 (and 8
for the prompt sharding alone, the bench's N = 8 layout: C = 10 prompts over 8 ranks).

The protocol — images sharded by rank, text prompts sharded with an all-gather of the features and
a SUM all-reduce of dL/dT, per-layer-group gradient buckets averaged at the end — is run with the
oracle (fp32 autograd, test infrastructure) as the per-rank compute, and the averaged PEFT
gradients must equal the single-process gradients of the global-mean loss over the whole batch
(the reference computes one loss over the gathered global batch)."""
import os
import socket
import sys
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "lifelong-clip_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from oracle import clip_oracle as o  # noqa: E402

B_GLOBAL = 4
C = 3  # not a multiple of the world size: exercises the prompt padding


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _inputs(method):
    cfg = o.TINY
    sd = o.synthetic_state_dict(cfg, method, "both", seed=11)
    img = o.synthetic_images(B_GLOBAL, cfg.image_resolution, seed=3)
    tok = o.synthetic_tokens(C, cfg.context_length, seed=4, vocab=cfg.vocab_size)
    y = torch.tensor([2, 0, 1, 2])
    return cfg, sd, img, tok, y


def _trainable(sd):
    vis, txt = o.tower_prefixes(o.TINY)
    names = [n for n in sd if o.is_trainable(n)]
    img_names = [n for n in names if n.startswith("visual.")]
    txt_names = [n for n in names if not n.startswith("visual.")]
    return img_names, txt_names


def _reference_grads(method):
    cfg, sd, img, tok, y = _inputs(method)
    _, _, _, _, grads, _ = o.train_step(img, tok, y, sd, cfg, method, "both")
    return grads


def _worker(rank, port, tmpdir, method, bucket_layers, WORLD):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    torch.set_num_threads(1)
    from lcclip.dp import DataParallel
    dp = DataParallel()
    assert dp.world == WORLD and dp.rank == rank
    cfg, sd, img, tok, y = _inputs(method)
    per_img = B_GLOBAL // WORLD
    img_l = img[rank * per_img:(rank + 1) * per_img]
    y_l = y[rank * per_img:(rank + 1) * per_img]
    leaves = {n: t.detach().clone().requires_grad_(o.is_trainable(n)) for n, t in sd.items()}
    img_names, txt_names = _trainable(sd)

    # forward: local images, this rank's prompt slice, gathered text features
    fi = o.encode_image(img_l, leaves, cfg, method, "both")
    tok_s = dp.shard_tokens(tok)
    lo, hi, per = dp.prompt_slice(C)
    assert tok_s.shape[0] == per
    ft_s = o.encode_text(tok_s, leaves, cfg, method, "both")
    ft_all = dp.gather_rows(ft_s.detach(), C).requires_grad_(True)
    assert ft_all.shape[0] == C
    logits, _, _ = o.clip_logits(fi, ft_all, leaves["logit_scale"])
    loss = o.loss_on_probs(logits.softmax(-1), y_l)  # local mean (DDP semantics)
    img_leaves = [leaves[n] for n in img_names]
    g_img = torch.autograd.grad(loss, img_leaves + [ft_all])
    d_t = g_img[-1]
    # dL/dT from every rank's images, SUMmed, then each rank backprops its own slice
    d_tp = torch.zeros(per * WORLD, d_t.shape[1])
    d_tp[:C] = d_t
    dp.sum_async(d_tp).wait()
    g_txt = torch.autograd.grad(ft_s, [leaves[n] for n in txt_names], grad_outputs=d_tp[lo:hi])

    # flat buffer: image params then text params; buckets as the trainer launches them
    flat = torch.cat([g.reshape(-1) for g in list(g_img[:-1]) + list(g_txt)])
    n_img = sum(g.numel() for g in g_img[:-1])
    # image layer buckets (uneven split on purpose), then the text range
    cuts = sorted(set([0, n_img // 3, n_img]))
    for a, b in zip(cuts[:-1], cuts[1:]):
        dp.launch_bucket(flat, a, b)
    dp.launch_bucket(flat, n_img, flat.numel())
    dp.finish_buckets(flat)
    torch.save({"flat": flat, "names": img_names + txt_names,
                "shapes": [tuple(leaves[n].shape) for n in img_names + txt_names]},
               os.path.join(tmpdir, f"rank{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("method,WORLD", [("lora", 2), ("adapter", 2), ("adapter", 4)])
def test_dp_protocol_matches_global_batch(method, WORLD):
    ref = _reference_grads(method)
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(_free_port(), tmp, method, 1, WORLD), nprocs=WORLD, join=True)
        outs = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(WORLD)]
    # every rank ends with the same averaged gradients
    for r in range(1, WORLD):
        assert torch.equal(outs[0]["flat"], outs[r]["flat"])
    flat = outs[0]["flat"]
    off = 0
    worst = 0.0
    for n, shp in zip(outs[0]["names"], outs[0]["shapes"]):
        k = 1
        for d in shp:
            k *= d
        g = flat[off:off + k].reshape(shp)
        off += k
        r = ref[n]
        err = ((g - r).norm() / r.norm().clamp_min(1e-30)).item()
        worst = max(worst, err)
        assert err < 1e-4, (n, err)
    assert off == flat.numel()
    assert set(outs[0]["names"]) == set(ref.keys())


def _slice_worker(rank, port, tmpdir, WORLD):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from lcclip.dp import DataParallel
    dp = DataParallel()
    res = {}
    for Cn in (1, 2, 5, 8, 10):
        tok = torch.arange(Cn * 4).reshape(Cn, 4)
        s = dp.shard_tokens(tok)
        lo, hi, per = dp.prompt_slice(Cn)
        feats = s.float() * 10
        full = dp.gather_rows(feats, Cn)
        res[Cn] = (s, full, (lo, hi, per))
    torch.save(res, os.path.join(tmpdir, f"s{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("WORLD", [2, 8])
def test_prompt_sharding_covers_every_prompt_once(WORLD):
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_slice_worker, args=(_free_port(), tmp, WORLD), nprocs=WORLD, join=True)
        outs = [torch.load(os.path.join(tmp, f"s{r}.pt"), weights_only=True) for r in range(WORLD)]
    for Cn in (1, 2, 5, 8, 10):
        tok = torch.arange(Cn * 4).reshape(Cn, 4)
        per = -(-Cn // WORLD)
        for r in range(WORLD):
            s, full, (lo, hi, p) = outs[r][Cn]
            assert p == per and (lo, hi) == (r * per, (r + 1) * per)
            # gathered features are exactly the per-prompt features, padding dropped
            assert torch.equal(full, tok.float() * 10)
            # a rank's slice is its rows of the list padded with copies of the last prompt
            padded = torch.cat([tok, tok[-1:].expand(per * WORLD - Cn, -1)], 0)
            assert torch.equal(s, padded[lo:hi])


def test_single_process_is_a_noop():
    from lcclip.dp import DataParallel
    dp = DataParallel()
    assert dp.world == 1 and dp.rank == 0
    assert dp.prompt_slice(7) == (0, 7, 7)
    t = torch.arange(5.)
    assert dp.sum_async(t) is None
    dp.launch_bucket(t, 0, 5)
    dp.finish_buckets(t)
    assert torch.equal(t, torch.arange(5.))
    tok = torch.arange(12).reshape(3, 4)
    assert torch.equal(dp.shard_tokens(tok), tok)


def _replica_worker(rank, port, tmpdir, WORLD):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from lcclip import AdapterCLIP, OnlineTrainer
    from test_surface import TINY_ARCH
    torch.manual_seed(1234 + 17 * rank)  # a rank-dependent draw: every rank builds other weights
    w = AdapterCLIP("tiny", peft_method="adapter", peft_encoder="both", arch_overrides=TINY_ARCH)
    w.set_token(torch.arange(2 * 77).reshape(2, 77) % 500 + rank)  # buffers differ too
    before = {k: v.detach().clone() for k, v in w.state_dict().items()}
    tr = OnlineTrainer(w, distributed=True)
    after = {k: v.detach().clone() for k, v in w.state_dict().items()}
    torch.save({"before": before, "after": after, "flat_p": tr.flat_p.clone()},
               os.path.join(tmpdir, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("WORLD", [2, 4])
def test_trainer_replicates_rank0_once(WORLD):
    """verdict r5: the ranks' replicas are made identical at trainer construction (the one-time
    form of DataParallel's per-step replicate, methods/_trainer.py:167-168), not by seeding
    alone: ranks built from different random draws all hold rank 0's parameters and buffers
    afterwards, PEFT views of the flat buffer included."""
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_replica_worker, args=(_free_port(), tmp, WORLD), nprocs=WORLD, join=True)
        outs = [torch.load(os.path.join(tmp, f"r{r}.pt"), weights_only=True) for r in range(WORLD)]
    r0 = outs[0]["before"]
    for r in range(1, WORLD):
        differ = [k for k in r0 if not torch.equal(outs[r]["before"][k], r0[k])]
        assert differ  # the ranks did start apart
        for k, v in r0.items():
            assert torch.equal(outs[r]["after"][k], v), (r, k)
        assert torch.equal(outs[r]["flat_p"], outs[0]["flat_p"])
    for k, v in r0.items():
        assert torch.equal(outs[0]["after"][k], v), k  # rank 0 keeps its own


def _module_dp_worker(rank, port, tmpdir, WORLD):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from lcclip.dp import ModuleDataParallel
    torch.manual_seed(100 + rank)  # rank-dependent init: replication must fix it
    net = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3))
    net.register_buffer("count", torch.zeros(3))
    net[0].bias.requires_grad_(False)  # a frozen parameter is replicated but not averaged
    ddp = ModuleDataParallel(net)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4 * WORLD, 6, generator=g)
    y = torch.randint(0, 3, (4 * WORLD,), generator=g)
    sl = slice(rank * 4, (rank + 1) * 4)
    loss = torch.nn.functional.cross_entropy(net(x[sl]), y[sl])
    loss.backward()
    ddp.sync_grads()
    num = y[sl].bincount(minlength=3).float()
    net.count += ddp.all_sum(num)
    classes = ddp.exposed_classes([int(c) for c in y[sl]][::-1])
    torch.save({"state": {k: v.clone() for k, v in net.state_dict().items()},
                "grads": {n: p.grad.clone() for n, p in net.named_parameters() if p.grad is not None},
                "classes": classes}, os.path.join(tmpdir, f"m{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("WORLD", [2, 4])
def test_module_data_parallel(WORLD):
    """lcclip.dp.ModuleDataParallel (the autograd surfaces' DDP, MVP / MaPLe): rank 0's weights
    and buffers replicated at construction, trainable gradients averaged to the global-batch
    gradient, per-batch counts summed, and the exposed-class list merged in rank order with the
    first occurrence kept (methods/mvp_clip.py:300-313)."""
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_module_dp_worker, args=(_free_port(), tmp, WORLD), nprocs=WORLD, join=True)
        outs = [torch.load(os.path.join(tmp, f"m{r}.pt"), weights_only=True) for r in range(WORLD)]
    # single process, global batch, rank 0's initial weights
    torch.manual_seed(100)
    net = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3))
    net[0].bias.requires_grad_(False)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4 * WORLD, 6, generator=g)
    y = torch.randint(0, 3, (4 * WORLD,), generator=g)
    torch.nn.functional.cross_entropy(net(x), y).backward()
    for r in range(WORLD):
        for n, p in net.named_parameters():
            if p.requires_grad:
                assert torch.allclose(outs[r]["grads"][n], p.grad, atol=1e-6), (r, n)
            else:
                assert n not in outs[r]["grads"]
        for k, v in net.state_dict().items():
            assert torch.equal(outs[r]["state"][k], v), (r, k)
        assert torch.equal(outs[r]["state"]["count"], y.bincount(minlength=3).float())
    want = []
    for r in range(WORLD):
        for c in [int(c) for c in y[r * 4:(r + 1) * 4]][::-1]:
            if c not in want:
                want.append(c)
    assert all(o_["classes"] == want for o_ in outs)
