"""Benchmark: one online-CL optimizer step (methods/adapter_clip.py:86-96) of CLIP ViT-B/16 +
12-layer text tower with adapters on both towers (BASELINE.json configs[1]: adapter_clip, bf16,
batch 256 per GPU, 1x MI355X), on synthetic 224x224 images and C = 10 class prompts.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--classes C]
                  [--method adapter|lora] [--no-cpu-baseline]

For N > 1 bench.py starts the N ranks itself (torch.distributed.run in a child process, one
process per GPU, RCCL over xGMI; launching it under torch.distributed.run works too); per-GPU work is fixed
(weak scaling): images shard by rank, the C prompts are sharded across ranks (features
all-gathered, dL/dT all-reduced), and the PEFT gradients are all-reduced in per-layer-group
buckets overlapped with backward (lcclip/dp.py).
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import math
import os
import sys
import time

# HIP hardware queues per process: at least 8 (lcclip's own rule, applied here too because HIP
# reads it when the runtime initialises, before lcclip is imported below; the GPU box exports
# HIP's default, 4): main, text-tower, weight-gradient and RCCL streams each on their own queue.
# Recorded in the output line. With fewer than 6 queues the trainer shares one side stream
# between the text tower and the PEFT weight gradients (OnlineTrainer._merge_side_streams), which
# costs 6-12 % (profiles/r05/b/).
def _raise_hw_queues(n=8):
    try:
        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
    except ValueError:
        cur = 0
    if cur < n:
        os.environ["GPU_MAX_HW_QUEUES"] = str(n)


_raise_hw_queues(int(os.environ.get("LCCLIP_HW_QUEUES", "8")))  # (A/B knob: the minimum)
HW_QUEUES = os.environ.get("GPU_MAX_HW_QUEUES")  # what HIP reads when it initialises below

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "lifelong-clip_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# Algorithmic FLOPs (fixed convention: frozen backbone, dX for all layers,
# attention core counted 3x in fwd+bwd).
F_IMG_FWD = 35.127e9
F_IMG = {"vanilla": 71.453e9, "lora": 71.714e9, "adapter": 74.242e9}
F_TXT = {"vanilla": 12.065e9, "lora": 12.065e9 + 0.068e9, "adapter": 12.065e9 + 0.727e9}
PEAK_BF16 = 2.5e15      # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, spec)
PEAK_HBM = 8.0e12


def synthetic_batch(B, C, dev, seed, tok_seed=7):
    """Images / labels from `seed` (per rank); the C prompts from `tok_seed` (the same global
    class list on every rank)."""
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.rand(B, 3, 224, 224, device=dev, generator=g)
    mean = torch.tensor([0.5071, 0.4867, 0.4408], device=dev).view(1, 3, 1, 1)
    std = torch.tensor([0.2675, 0.2565, 0.2761], device=dev).view(1, 3, 1, 1)
    x = (x - mean) / std
    gc = torch.Generator().manual_seed(tok_seed)
    tok = torch.zeros(C, 77, dtype=torch.long)
    for i in range(C):
        k = int(torch.randint(6, 13, (1,), generator=gc))
        tok[i, 0] = 49406
        tok[i, 1:1 + k] = torch.randint(256, 49406, (k,), generator=gc)
        tok[i, 1 + k] = 49407
    y = torch.randint(0, C, (B,), generator=torch.Generator().manual_seed(seed))
    return x, tok.to(dev), y.to(dev)


def routes_to_blaslt(M, N, K, epi, bias, alpha, dtype):
    """lc_gemm_nt_ex's hipBLASLt route (gemm.hip, blaslt.hip): the plain bf16 QKV input-gradient
    GEMM of a 256-image step (M >= 32 768, N = 768, K = 2 304, no epilogue, no bias)."""
    return (dtype == torch.bfloat16 and epi == 0 and bias is None and alpha == 1.0
            and M >= 32768 and N == 768 and K == 2304)


def routes_to_pp(M, N, K, epi, cus=256):
    """The lc_gemm_nt tile selector's rule for the 256x256 phase-interleaved kernel (gemm.hip,
    lc_gemm_nt_ex -> gemm8_kernel): the dominant kernel of the step."""
    if N % 256 or M < 4096 or K <= 64:
        return False
    t256 = (M + 255) // 256 * (N // 256)
    full, rem = divmod(t256, cus)
    tail_ok = full >= 2 or rem == 0 or 2 * rem >= cus or (2 * rem <= cus and K >= 1024)
    return (t256 >= cus and tail_ok) or (2 * t256 >= cus and K >= 2048)


class GemmTimer:
    """Times every lc_gemm_nt launch of one step with HIP events on the launch stream (torch's
    current stream, which ops.gemm_nt launches on) and sums the algorithmic FLOPs (2*M*N*K) and
    algorithmic HBM bytes (A, B, outputs and side inputs once each) of the launches that route
    to the ping-pong kernel."""

    def __init__(self, ops_mod):
        self.ops = ops_mod
        self.orig = ops_mod.gemm_nt
        self.records = []

    def __enter__(self):
        main = torch.cuda.current_stream()

        def timed(A, B, epi, out0, **kw):
            st = torch.cuda.current_stream()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(st)
            r = self.orig(A, B, epi, out0, **kw)
            e1.record(st)
            M, K = A.shape
            N = B.shape[0]
            nbytes = (M * K + N * K) * 2 + out0.numel() * out0.element_size()
            for extra in ("out1", "aux"):
                t = kw.get(extra)
                if t is not None:
                    nbytes += t.numel() * t.element_size()
            lib = routes_to_blaslt(M, N, K, epi, kw.get("bias"), kw.get("alpha", 1.0), A.dtype)
            self.records.append((e0, e1, 2.0 * M * N * K, nbytes,
                                 routes_to_pp(M, N, K, epi) and not lib, st == main, lib))
            return r
        self.ops.gemm_nt = timed
        import lcclip.engine as eng
        eng.ops.gemm_nt = timed
        return self

    def __exit__(self, *a):
        self.ops.gemm_nt = self.orig

    def summary(self):
        """Sums over the step's GEMM launches. `pp_*`: the dominant-kernel launches on the main
        (image-chain) stream only — side-stream launches (text tower, PEFT weight gradients) run
        concurrently with them, so their durations are reported apart (`side_ms`) and never summed
        into a share of the step."""
        torch.cuda.synchronize()
        main = [r for r in self.records if r[5]]
        ms = sum(r[0].elapsed_time(r[1]) for r in main)
        side_ms = sum(r[0].elapsed_time(r[1]) for r in self.records if not r[5])
        pp = [(r[0].elapsed_time(r[1]), r[2], r[3]) for r in main if r[4]]
        lib = [(r[0].elapsed_time(r[1]), r[2]) for r in main if r[6]]
        return dict(n=len(main), ms=ms, side_n=len(self.records) - len(main), side_ms=side_ms,
                    pp_n=len(pp), pp_ms=sum(t for t, _, _ in pp),
                    pp_flops=sum(f for _, f, _ in pp), pp_bytes=sum(b for _, _, b in pp),
                    lib_n=len(lib), lib_ms=sum(t for t, _ in lib), lib_flops=sum(f for _, f in lib))


class TowerTimer:
    """HIP events (torch's current stream, where the image tower launches) around the image
    tower's forward and backward of every step of the timed loop: the SURVEY §8(d) north-star
    ratio B * F_img / (t_image_tower * peak), text tower and head excluded. The backward span
    ends after the side-stream PEFT weight gradients have joined (they are image-tower work).
    Events are recorded inside the back-to-back loop that `value` times (no synchronize before
    a step), so a step's tower time is its share of that loop; the median over steps is reported."""

    def __init__(self, tower):
        self.tower = tower
        self.spans = []

    def __enter__(self):
        self.fwd, self.bwd = self.tower.forward, self.tower.backward

        def wrap(fn):
            def timed(*a, **kw):
                st = torch.cuda.current_stream()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(st)
                r = fn(*a, **kw)
                e1.record(st)
                self.spans.append((e0, e1))
                return r
            return timed
        self.tower.forward, self.tower.backward = wrap(self.fwd), wrap(self.bwd)
        return self

    def __exit__(self, *a):
        self.tower.forward, self.tower.backward = self.fwd, self.bwd

    def ms(self):
        """Per-step tower time (fwd + bwd spans; two spans per step), median over the steps."""
        torch.cuda.synchronize()
        per = [self.spans[i][0].elapsed_time(self.spans[i][1]) +
               self.spans[i + 1][0].elapsed_time(self.spans[i + 1][1])
               for i in range(0, len(self.spans) - 1, 2)]
        if not per:
            return None
        per.sort()
        return per[len(per) // 2]


def pmc_traffic():
    """HBM bytes per launch of the dominant GEMM family from the latest committed PMC summary
    (tools/profile_round.sh + tools/pmc_traffic.py), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "gemm_traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    fam = d.get("families", {}).get("gemm8_kernel_bf16")
    if not fam:
        return None, None
    return fam["bytes_per_launch"], os.path.relpath(files[-1], ROOT)


def time_train_transform(B, dev, reps=20):
    """The GPU train transform (lcclip.transforms) on a CIFAR-shaped batch,
    fused into conv1's patch layout: average launch time with HIP events on its stream, and the
    HBM rate of its algorithmic bytes (input f32 32x32 images + bf16 patch rows written).
    Reported beside the step; not part of `value`."""
    from lcclip.transforms import TrainTransform
    x = torch.randint(0, 256, (B, 3, 32, 32), device=dev).float() / 255
    tf = TrainTransform.for_dataset("cifar100", generator=torch.Generator().manual_seed(0))
    # a fixed two-op CIFAR10 sub-policy (AutoAugment kernel + resize/crop/flip/normalise kernel)
    prm = ([("Equalize", 0.0), ("Rotate", 20.0)], 4, 4, True)
    out = tf(x, params=prm, layout="patches")
    st = torch.cuda.current_stream(dev)

    def avg_us(p):
        tf(x, params=p, layout="patches")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            tf(x, params=p, layout="patches")
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3
    us = avg_us(prm)
    us_tf = avg_us((4, 4, True))  # no sub-policy: the resize/crop/flip/normalise kernel alone
    nbytes = x.numel() * 4 * 3 + out.numel() * 2  # autoaug read + write, transform read; output
    tf_bytes = x.numel() * 4 + out.numel() * 2
    return {"kernel": "autoaug_kernel (uint8 quantise + Equalize + Rotate) then "
                      "train_transform_sep_kernel (resize 32->224 + pad-crop + flip + normalise, "
                      "written as conv1 bf16 patch rows)",
            "batch": B, "avg_launch_us": round(us, 2), "algorithmic_bytes": nbytes,
            "transform_only_us": round(us_tf, 2),
            "transform_only_GBps": round(tf_bytes / (us_tf * 1e-6) / 1e9, 1),
            "achieved_GBps": round(nbytes / (us * 1e-6) / 1e9, 1), "peak_GBps": PEAK_HBM / 1e9}


def host_cores():
    """(cores to use, os.cpu_count(), cgroup CPU quota in cores or None). SURVEY §8(d) asks for
    os.cpu_count() threads; on a shared GPU box the process's cgroup may grant fewer CPUs than
    the machine has (oversubscribing them only slows the baseline down), so the thread count is
    os.cpu_count() capped by the affinity mask and the cgroup quota, all three reported."""
    n_all = os.cpu_count() or 1
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else n_all
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except Exception:
        pass
    if quota is not None:
        n = min(n, quota)
    return max(1, min(n, n_all)), n_all, quota


def cpu_baseline(seconds_cap=60.0, warmup=2, timed=5):
    """The oracle (fp32 PyTorch-CPU restatement, oracle/clip_oracle.py) at BASELINE config 1:
    LoRA both towers, B = 16, C = 16, one full step (fwd, CE-on-probs, bwd, AdamW), timed as
    SURVEY §8(d) says: 2 warm-up + 5 timed steps (fewer timed steps only if the cap is hit)."""
    from oracle import clip_oracle as o
    threads, n_all, quota = host_cores()
    torch.set_num_threads(threads)
    cfg = o.VIT_B16
    sd = o.synthetic_state_dict(cfg, "lora", "both", seed=1234)
    img = o.synthetic_images(16, 224, seed=0)
    tok = o.synthetic_tokens(16, 77, seed=0)
    y = torch.randint(0, 16, (16,), generator=torch.Generator().manual_seed(0))
    t_start = time.time()
    for _ in range(warmup):
        o.train_step(img, tok, y, sd, cfg, "lora", "both")
    times = []
    while len(times) < timed and (not times or time.time() - t_start + times[-1] < seconds_cap):
        t0 = time.time()
        o.train_step(img, tok, y, sd, cfg, "lora", "both")
        times.append(time.time() - t0)
    times.sort()
    med = times[len(times) // 2]
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = "unknown"
    return {"value": round(16 / med, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "host_cpu_count": n_all, "cgroup_cpu_quota": quota,
            "sample": f"oracle fp32 train step, ViT-B/16+text LoRA both towers, B=16, C=16, "
                      f"median of {len(times)} timed steps after {warmup} warm-up, "
                      f"{threads} threads ({model})"}


def visible_gpu_count():
    """GPUs this job may use, asked in a child process so that the launching parent never
    touches the GPU (the ranks it starts must be the first processes to initialise HIP)."""
    import subprocess
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        raise SystemExit(f"bench.py: could not count GPUs (rc {r.returncode}): {r.stderr[-400:]}")


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(n, argv, port):
    """One process per GPU on this node through torch.distributed.run (it sets RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR/PORT for each rank; rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__), *argv]


def launch_ranks(n, argv, gpu_count=visible_gpu_count, run=None):
    """`bench.py --gpus N` started without a launcher (WORLD_SIZE unset): start the N ranks as
    child processes and return the launcher's exit status (non-zero if any rank failed). This
    replaces the reference's single-process `nn.DataParallel` (methods/_trainer.py:132, 167-168)
    with one RCCL rank per GPU. The parent makes no GPU call: it only counts the devices in a
    child, refuses a job larger than the node, and waits."""
    import subprocess
    have = gpu_count()
    if have < n:
        raise SystemExit(f"bench.py --gpus {n}: only {have} GPU(s) visible on this node")
    cmd = launch_cmd(n, argv, free_port())
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return (run or subprocess.call)(cmd, env=env)


def main():
    if "WORLD_SIZE" not in os.environ:
        pre = argparse.ArgumentParser(add_help=False)
        pre.add_argument("--gpus", type=int, default=1)
        pre.add_argument("--force-dist", action="store_true")
        a, _ = pre.parse_known_args()
        if a.gpus < 1:
            raise SystemExit("--gpus must be >= 1")
        if a.gpus > 1 or a.force_dist:
            sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--method", default="adapter", choices=["adapter", "lora", "vanilla"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the RCCL process group and the DP exchange even at N=1 "
                         "(exercises the collective path; launch through torch.distributed.run)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as a HIP graph (1 GPU; measured equal to eager at B=256)")
    ap.add_argument("--text-precision", default="fp16", choices=["fp16", "bf16"],
                    help="the text tower's 16-bit storage (AdapterCLIP text_precision)")
    ap.add_argument("--image-precision", default="bf16", choices=["bf16", "fp16"],
                    help="the image tower's 16-bit storage (AdapterCLIP image_precision): bf16 is "
                         "BASELINE config 2's; fp16 is the reference's autocast arithmetic "
                         "(a parity mode, reported beside the bf16 headline)")
    ap.add_argument("--gemm-tile", type=int, default=0,
                    help="A/B knob: lc_gemm_set_tile value for every GEMM (0 = automatic)")
    ap.add_argument("--streamk", type=int, default=None,
                    help="A/B knob: lc_gemm_set_streamk mode (0 off, 1 N=768 K>=2048, 2 N=768, "
                         "3 every ragged 256x256 launch; default: the library's)")
    ap.add_argument("--attn-bwd-form", type=int, default=None,
                    help="A/B knob: lc_attn_bwd_set_form (1 fused dS^T park, 2 split pair, "
                         "3 two-phase at two workgroups per CU; default: the library's)")
    ap.add_argument("--peft-encoder", default=None, choices=["both", "image", "text", "none"],
                    help="which towers carry the PEFT residuals (AdapterCLIP peft_encoder; default "
                         "both, config 2's; 'image' freezes the text tower, whose features are "
                         "then cached across steps: a measurement of the text tower's cost)")
    ap.add_argument("--resid32", action="store_true",
                    help="A/B knob: the image tower's residual stream in f32 instead of IEEE half")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dp = world > 1 or args.force_dist
    if args.force_dist:
        os.environ["LCCLIP_DP_FORCE"] = "1"  # lcclip.dp: collectives even on a one-rank group
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}")
    if dp:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
        world = dist.get_world_size()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from lcclip import AdapterCLIP, OnlineTrainer, ops
    if args.gemm_tile:
        from lcclip import _lib
        if _lib.load().lc_gemm_set_tile(args.gemm_tile) != 0:
            raise SystemExit(f"--gemm-tile {args.gemm_tile} rejected")
    if args.streamk is not None:
        from lcclip import _lib
        if _lib.load().lc_gemm_set_streamk(args.streamk) != 0:
            raise SystemExit(f"--streamk {args.streamk} rejected")
    if args.attn_bwd_form is not None:
        from lcclip import _lib
        if _lib.load().lc_attn_bwd_set_form(args.attn_bwd_form) != 0:
            raise SystemExit(f"--attn-bwd-form {args.attn_bwd_form} rejected")
    if args.resid32:
        from lcclip.engine import ImageTower
        ImageTower.RESID16 = False
    torch.manual_seed(1234)  # identical random-init weights on every rank
    peft = "both" if args.method != "vanilla" else "none"
    if args.peft_encoder is not None:
        peft = args.peft_encoder
    model = AdapterCLIP("ViT-B/16", peft_method=args.method, peft_encoder=peft, device=dev,
                        text_precision=args.text_precision, image_precision=args.image_precision)
    trainer = OnlineTrainer(model, distributed=dp,
                            shard_text=os.environ.get("LCCLIP_DP_NOSHARD") != "1",
                            overlap_text=os.environ.get("LCCLIP_OVERLAP_TEXT", "1") != "0",
                            overlap_grads=os.environ.get("LCCLIP_OVERLAP_GRADS", "1") != "0")
    B, C = args.batch, args.classes
    x, tok, y = synthetic_batch(B, C, dev, seed=100 + rank)
    graph = trainer.enable_graph(x, y, tok) if args.graph else False

    for _ in range(args.warmup):
        trainer.step(x, y, tok)
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    torch.cuda.synchronize()
    with TowerTimer(trainer.img) as tt:
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss, probs = trainer.step(x, y, tok)
        torch.cuda.synchronize()
        if dp:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev)
    if dp:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = t.item()
    ms = dt / args.steps * 1e3
    total_ips = world * B * args.steps / dt

    # dominant kernel (lc_gemm_nt family) timed live with HIP events on its launch stream,
    # over one extra, untimed step
    with GemmTimer(ops) as gt:
        trainer.eager_step(x, y, tok)
    gs = gt.summary()
    img_ms = tt.ms()
    img_src = "timed loop"
    if img_ms is None:  # graph replay: the tower's methods are not called per step
        with TowerTimer(trainer.img) as tt2:
            trainer.eager_step(x, y, tok)
            trainer.eager_step(x, y, tok)
        img_ms, img_src = tt2.ms(), "eager steps after the timed loop (graph mode)"
    tf_stats = time_train_transform(B, dev)

    if rank == 0:
        f_img = F_IMG[args.method]
        f_step = B * f_img + C * F_TXT[args.method] + 6 * B * C * 512
        achieved = gs["pp_flops"] / (gs["pp_ms"] * 1e-3)
        traffic, traffic_src = pmc_traffic()
        n_pp = max(gs["pp_n"], 1)
        out = {
            "metric": "images/sec/GPU (ViT-B/16 fwd+bwd, bs=256) + online A_AUC on CIFAR-100",
            "metric_note": "value is the throughput half only; A_AUC needs CIFAR-100 and CLIP "
                           "weights (absent offline) - the online loop that computes it "
                           "(lcclip.online) is exercised on synthetic data in the tests",
            "value": round(total_ips, 2),
            "unit": "images/s",
            "n_gpus": world,
            "rccl_world": dist.get_world_size() if dp else None,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"bf16": "bf16", "fp16": "f16"}[args.image_precision],
            "text_tower_dtype": {"fp16": "f16", "bf16": "bf16"}[args.text_precision],
            # the image tower's residual stream (the reference's autocast dtype: fp16)
            "image_residual_dtype": "f16" if trainer.img._resid16() else "f32",
            # and its gradient (fp16 under a per-call power-of-two scale: the GradScaler's role)
            "image_residual_grad_dtype": "f16" if (
                trainer.img._resid16() and trainer.img.HALF_GRAD and (
                    trainer.img.stack.variant == "adapter" or (
                        trainer.img.stack.variant == "lora"
                        and trainer.img.stack.lora_half_grad_ok()))) else "f32",
            "data": "synthetic (random-init ViT-B/16 CLIP weights, U[0,1) images normalised with "
                    "CIFAR-100 stats, random prompt token ids)",
            "config": {"workload": f"{args.method}_clip ViT-B/16 "
                                   f"{'both towers' if peft == 'both' else 'peft_encoder=' + peft}, online_train step "
                                   f"(fwd + CE-on-probs + bwd + AdamW)",
                       "global_batch": B * world, "per_gpu_batch": B, "seq_len": 197,
                       "text_prompts": C, "parallelism": f"dp{world}",
                       "launch": "hip_graph" if graph else "eager"},
            "images_per_s_per_gpu": round(total_ips / world, 2),
            "mfma_frac_step": round(f_step / (ms * 1e-3) / PEAK_BF16, 4),
            "image_tower": {"ms_fwd_bwd": round(img_ms, 3),
                            "tflops": round(B * f_img / (img_ms * 1e-3) / 1e12, 1),
                            "mfma_frac": round(B * f_img / (img_ms * 1e-3) / PEAK_BF16, 4),
                            "mfma_frac_step_bound": round(B * f_img / (ms * 1e-3) / PEAK_BF16, 4),
                            "flops_per_image": f_img,
                            "source": img_src,
                            "note": "SURVEY 8(d) north-star ratio: B*F_img / (t_image_tower * "
                                    "peak), t = median over the timed steps of the HIP-event "
                                    "spans around the tower's fwd and bwd on the main stream; "
                                    "mfma_frac_step_bound = the same with the whole step time "
                                    "(a lower bound of mfma_frac)"},
            "roofline": {"bound": "mfma",
                         "kernel": "gemm8_kernel<EPI 0|2|6|7, bf16> (256x256 phase-interleaved "
                                   "bf16 MFMA GEMM: QKV, out-proj, c_fc+QuickGELU+QuickGELU', "
                                   "c_proj fwd; out-proj, c_fc, c_proj dX)",
                         "achieved": round(achieved / 1e12, 2), "peak": PEAK_BF16 / 1e12,
                         "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_unit": "bytes per launch (PMC FETCH_SIZE*2 + WRITE_SIZE)",
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": round(gs["pp_bytes"] / n_pp),
                         "flops_per_launch": round(gs["pp_flops"] / n_pp),
                         "launches_per_step": gs["pp_n"],
                         "avg_launch_ms": round(gs["pp_ms"] / n_pp, 4),
                         "main_stream_gemm_share_of_step": round(gs["ms"] / ms, 3),
                         "side_stream_gemm_ms": round(gs["side_ms"], 3),
                         "note": "launches of the dominant kernel on the main (image-chain) "
                                 "stream, timed with HIP events around each launch of one extra "
                                 "eager step"},
            # the one plain GEMM the library routes to hipBLASLt (QKV dX at 256 images), apart
            "library_gemm": {"kernel": "hipBLASLt (QKV input gradient, plain bf16 GEMM)",
                             "launches_per_step": gs["lib_n"],
                             "avg_launch_ms": round(gs["lib_ms"] / max(gs["lib_n"], 1), 4),
                             "tflops": round(gs["lib_flops"] / max(gs["lib_ms"], 1e-9) / 1e9, 1)},
            "runtime": {"GPU_MAX_HW_QUEUES": HW_QUEUES,
                        "side_streams": 1 if trainer._merge_side_streams() else 2,
                        "side_stream_cus": trainer.side_cus},
            "train_transform": tf_stats,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), flush=True)
    if dp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
