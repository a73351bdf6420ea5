#!/usr/bin/env python3
"""Flagship benchmark: task.py-style DDP training throughput (samples/sec, whole node).

BASELINE.json metric: "samples/sec (whole node) task.py DDP at 1/2/4/8 MI355X; scaling
efficiency"; config: ResNet-50, ImageNet shape (3x224x224, 1000 classes), 256 images per GPU
(weak scaling), bf16 compute with fp32 master weights, SGD(lr=0.1, momentum=0.9, wd=1e-4)
exactly as task.py:212-214, synthetic data generated on the device, random-init weights.

One timed step = zero_grad + forward + cross-entropy + backward (with the bucketed RCCL
gradient all-reduce overlapped) + optimizer step — the reference hot loop (task.py:308-312).
W untimed warmup steps, then exactly K steps bracketed by barrier + device sync on both
sides; the reported time is the MAX over ranks.

Single GPU:   python bench.py --gpus 1 --steps 20 --warmup 5
Multi GPU:    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
                  --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W
          or  python bench.py --gpus N ...   (no WORLD_SIZE in the env: this process spawns the
              N rank processes itself before anything touches HIP — task.py:117-124's mp.spawn —
              and every rank checks that the process group really has N members)

The training step is replayed from a captured hipGraph on 1 GPU AND under DDP: the bucket
all-reduces (RCCL) and the per-forward buffer broadcast are captured into the same graph on
the process group's stream, so their overlap with backward survives replay.
``--force-reduce`` runs the whole DDP/RCCL path at world size 1 (profiling the collectives
on a one-GPU box); ``--device cpu`` runs the same harness on gloo (CPU tests).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "samples/sec (whole node) task.py DDP at 1/2/4/8 MI355X; scaling efficiency"
# Measured comparators: stock PyTorch-ROCm 2.10 (MIOpen + hipBLASLt, channels_last,
# bf16 autocast, torch SGD) on ONE MI355X, ResNet-50 b256 224x224: 6580.1 samples/s.
# vs_baseline = value / (comparator_per_gpu * n_gpus)  (ideal linear scaling of the comparator).
# BERT-base MLM (B=32 x S=128 / B=8 x S=512 per GPU, AdamW fused, SDPA, bf16 autocast): stock
# torch measured on the same MI355X with tools/gpu_bert.sh / gpu_prof_bert.sh.
STOCK_1GPU = {"resnet50": 6580.1, "resnet18_32": 76880.3, "resnet18_32_fp32": 76305.2,
              "bert_base_128": 2184.8, "bert_base_512": 540.8}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch (weak scaling); default 256 images / 32 sequences")
    ap.add_argument("--seq", type=int, default=128, help="BERT sequence length")
    ap.add_argument("--res", type=int, default=224)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--bucket-cap-mb", type=float, default=32.0)
    ap.add_argument("--comm-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="DDP gradient wire format (bf16: packed pre-scaled by 1/world, half the "
                         "all-reduce bytes; fp32 = the reference's)")
    ap.add_argument("--impl", default="mipipe", choices=["mipipe", "stock"],
                    help="stock = torch DDP + MIOpen comparator")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the whole training step (incl. DDP collectives) from a captured "
                         "hipGraph; auto = on when safe (SGD, no dropout)")
    ap.add_argument("--force-reduce", action="store_true",
                    help="wrap in DDP and issue every collective even at world size 1")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = gloo backend, fp32 (harness tests without a GPU)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"],
                    help="compute dtype of the mipipe kernels (fp32 = the reference's precision)")
    ap.add_argument("--deterministic", type=int, default=0,
                    help="1: fixed-order reductions (no float atomics), bit-reproducible steps")
    ap.add_argument("--tune", type=int, default=1,
                    help="1: autotune conv tile configs per shape in the warm-up (cudnn.benchmark "
                         "analogue; in deterministic mode only a loaded / shipped table is used); "
                         "0: heuristic tile choice; 2: time candidates even in deterministic mode "
                         "(to build a shipped table with --save-tune)")
    ap.add_argument("--bert-dropout", type=float, default=None,
                    help="BERT hidden / attention dropout (default: the model's 0.1)")
    ap.add_argument("--emulate-ranks", type=int, default=1,
                    help="world-1 reference for DDP equivalence tests: every step runs the R "
                         "per-rank batches one after another (each BN sees its own chunk, rank 0's "
                         "buffers are kept, as DDP's per-forward broadcast does) and averages "
                         "their gradients before one optimizer step")
    ap.add_argument("--dump-params", default=None,
                    help="directory: each rank saves its final parameters and buffers there")
    ap.add_argument("--save-tune", default=None,
                    help="write the tuning table after the warm-up steps (JSON)")
    ap.add_argument("--reference-config", default="auto", choices=["auto", "on", "off"],
                    help="also time the reference's config of record in the same process "
                         "(ResNet-18 32x32, 1000 classes, fp32, deterministic, --ref-batch per "
                         "GPU) and report it as 'reference_config' in the JSON line; auto = with "
                         "the default mipipe ResNet-50 headline on the GPU")
    ap.add_argument("--time-deterministic", default="auto", choices=["auto", "on", "off"],
                    help="also time the headline in deterministic mode (the reference's "
                         "cudnn.deterministic=True, task.py:25) and report it as "
                         "'deterministic_variant'; auto = together with the reference config")
    ap.add_argument("--ref-batch", type=int, default=1024,
                    help="per-process batch of the reference config (task.py:58,153: 1024)")
    return ap.parse_args()


def _heartbeat(every_s: float = 30.0) -> None:
    """Progress line on stderr while a long step runs (first-call kernel compilation of stock
    MIOpen convs can take minutes)."""
    import threading

    def beat():
        t0 = time.time()
        while True:
            time.sleep(every_s)
            print(f"bench alive {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def _transports(path):
    if path is None:
        return None
    from mipipe.parallel.dist_utils import rccl_transports
    try:
        return rccl_transports(path)
    except OSError:
        return None


def _sync(dev) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def main() -> int:
    a = parse()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        # launched as `python bench.py --gpus N`: become the launcher (no HIP call so far)
        from mipipe.launch.local import spawn_local_ranks
        return spawn_local_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                 a.gpus)
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks",
              file=sys.stderr)
        return 2
    cpu = a.device == "cpu"
    if cpu:
        dev = torch.device("cpu")
    else:
        from mipipe.launch.env import device_offset
        local += device_offset()  # all GPUs visible, the launcher names this rank's (launch/env.py)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    distributed = world > 1 or a.force_reduce
    rccl_log = None
    if distributed:
        from mipipe.parallel.dist_utils import configure_rccl_env, enable_rccl_transport_log
        configure_rccl_env()  # high-priority RCCL stream: bucket all-reduces overlap backward
        if not cpu and world > 1:
            rccl_log = enable_rccl_transport_log()  # which transport each peer pair gets
        if cpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        if dist.get_world_size() != a.gpus:
            print(f"bench.py rank {rank}: process group has {dist.get_world_size()} ranks, "
                  f"expected {a.gpus}", file=sys.stderr)
            return 3
    a.distributed = distributed
    if rank == 0:
        _heartbeat()
    r = _run(a, world, rank, local, dev, distributed, cpu)
    det = None
    rd = None
    if _want_det_variant(a, cpu):
        # the headline again in the reference's own mode (task.py:25 cudnn.deterministic=True:
        # no float atomics, fixed-order reductions, shipped plan tables), same discipline
        import copy
        b = copy.copy(a)
        b.deterministic, b.dump_params, b.save_tune = 1, None, None
        del r["model"]
        if not cpu:
            torch.cuda.empty_cache()
        rd = _run(b, world, rank, local, dev, distributed, cpu)
        det = {"value": round(rd["value"], 2), "unit": "samples/s",
               "ms_per_step": round(rd["dt"] / b.steps * 1e3, 3), "steps": b.steps,
               "warmup": b.warmup, "deterministic": True,
               "hip_graph": bool(getattr(b, "graph_used", False)), "final_loss": rd["loss"],
               "cost_vs_default_pct": round(100.0 * (rd["dt"] / r["dt"] - 1.0), 2),
               "source": "task.py:25"}
    ref = None
    if _want_reference_config(a, cpu):
        # the reference's own config of record in the same process, same timing discipline:
        # ResNet-18 on 32x32 (CIFAR shape), 1000-class head (task.py:171), 1024 images per
        # process (task.py:153), fp32 (task.py:303-312: no autocast), deterministic kernels
        # (task.py:25: cudnn.deterministic = True)
        import copy
        b = copy.copy(a)
        b.model, b.res, b.classes, b.dtype, b.deterministic = "resnet18", 32, 1000, "fp32", 1
        b.batch = a.ref_batch
        b.emulate_ranks, b.dump_params, b.save_tune = 1, None, None
        r.pop("model", None)
        if rd is not None:  # the deterministic variant's DDP model and buckets: gone too
            rd.pop("model", None)
        if not cpu:
            torch.cuda.empty_cache()
        rr = _run(b, world, rank, local, dev, distributed, cpu)
        ref = {"model": "resnet18", "image_size": 32, "classes": 1000,
               "batch_per_gpu": b.batch, "global_batch": b.batch * world,
               "dtype": "fp32", "deterministic": True, "steps": b.steps, "warmup": b.warmup,
               "value": round(rr["value"], 2), "unit": "samples/s",
               "ms_per_step": round(rr["dt"] / b.steps * 1e3, 3),
               "vs_stock_fp32": (round(rr["value"] / (STOCK_1GPU["resnet18_32_fp32"] * world), 4)
                                 if not cpu else None),
               "hip_graph": bool(getattr(b, "graph_used", False)),
               "final_loss": rr["loss"], "gpu_clocks": rr["clocks"],
               "source": "task.py:25,153,171,212-214,303-312"}
    value, dt = r["value"], r["dt"]
    is_bert = a.model.startswith("bert")
    if is_bert:
        key = f"{a.model}_{a.seq}"
        opt_s = "AdamW(lr=1e-4,wd=0.01)"
    else:
        key = a.model if a.res == 224 else f"{a.model}_{a.res}"
        if a.dtype == "fp32":
            key += "_fp32"
        opt_s = "SGD(lr=0.1,momentum=0.9,wd=1e-4)"
    base = STOCK_1GPU.get(key)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "samples/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / (base * world), 4) if base else None,
            "dtype": "fp32" if (cpu or a.dtype == "fp32") else "bf16",
            "data": "synthetic (on-device, random-init weights)",
            "config": {"model": a.model, "global_batch": a.batch * world,
                       "seq_len": a.seq if is_bert else None,
                       "image_size": None if is_bert else a.res, "batch_per_gpu": a.batch,
                       "parallelism": f"dp{world}", "impl": a.impl, "optimizer": opt_s,
                       "hip_graph": bool(getattr(a, "graph_used", False)),
                       "deterministic": bool(a.deterministic),
                       "force_reduce": bool(a.force_reduce),
                       "comm_dtype": a.comm_dtype,
                       "native_reducer": bool(r.get("native_reducer", False)),
                       "rccl": _rccl_settings() if distributed else None,
                       "rccl_transports": _transports(rccl_log)},
            "final_loss": r["loss"], "gpu_clocks": r["clocks"]}
        if det is not None:
            line["deterministic_variant"] = det
        if ref is not None:
            line["reference_config"] = ref
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def _want_det_variant(a, cpu: bool) -> bool:
    if a.time_deterministic == "off" or a.deterministic:
        return False
    if a.time_deterministic == "on":
        return True
    return _want_reference_config(a, cpu) and a.reference_config != "off"


def _want_reference_config(a, cpu: bool) -> bool:
    if a.reference_config == "off":
        return False
    if a.reference_config == "on":
        return True
    # auto: alongside the default headline (mipipe ResNet-50) on the GPU
    return (not cpu and a.impl == "mipipe" and a.model == "resnet50" and a.emulate_ranks == 1
            and not a.dump_params)


def _run(a, world, rank, local, dev, distributed, cpu):
    """Build one config, W untimed warm-up steps, then exactly K timed steps bracketed by a
    barrier + device sync on both sides; the time is the MAX over ranks."""
    torch.manual_seed(0)
    if not cpu and a.impl == "mipipe":
        # per-shape conv tile autotuning during the (untimed, eager) warm-up steps — the
        # analogue of the reference's cudnn.benchmark = True (task.py:244)
        from mipipe.ops import tuning
        if a.deterministic:
            # a deterministic run takes its plans from the shipped / loaded tables only, never
            # from an earlier run's timing-based picks (bit-reproducible across processes)
            tuning.clear()
        tuning.from_env(bool(a.deterministic))
        tuning.set_benchmark(a.tune > 0, verbose=False, force=a.tune == 2)
        from mipipe.ops import determinism
        determinism.set_deterministic(bool(a.deterministic))

    is_bert = a.model.startswith("bert")
    if a.batch is None:
        a.batch = 32 if is_bert else 256
    if is_bert:
        step, model, batches = build_bert(a, world, local, dev, rank)
    else:
        step, model, batches = build_cnn(a, world, local, dev, rank)

    model.train()
    for i in range(a.warmup):
        loss = step(*batches[i % 2])
        if rank == 0:  # progress for long first steps (kernel autotuning, graph capture)
            print(f"warmup step {i + 1}/{a.warmup} ({a.model})", file=sys.stderr, flush=True)
    _sync(dev)
    if a.save_tune and rank == 0:
        from mipipe.ops import tuning
        tuning.save(a.save_tune)
    if distributed:
        dist.barrier()
    _sync(dev)
    from mipipe.obs.clocks import ClockSampler
    sampler = ClockSampler(local if not cpu else -1)
    if cpu:
        sampler.dir = None
    with sampler:  # sysfs reads on a daemon thread: shader clock / power during the timed steps
        t0 = time.perf_counter()
        for i in range(a.steps):
            loss = step(*batches[i % 2])
        _sync(dev)
        if distributed:
            dist.barrier()
        _sync(dev)
        dt = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        if hasattr(model, "check_comm_errors"):
            model.check_comm_errors(final=True)  # a one-shot wait that gave up fails the run
    if a.dump_params:
        inner = getattr(model, "module", model)
        os.makedirs(a.dump_params, exist_ok=True)
        torch.save({"params": [p.detach().cpu() for p in inner.parameters()],
                    "buffers": [b.detach().cpu() for b in inner.buffers()]},
                   os.path.join(a.dump_params, f"rank{rank}.pt"))
    return {"value": a.batch * world * a.steps / dt, "dt": dt,
            "loss": float(loss.detach().float().item()), "clocks": sampler.summary(),
            "native_reducer": bool(getattr(model, "native_reducer", False)), "model": model}


def build_bert(a, world, local, dev, rank):
    """BERT-base MLM: B sequences of S tokens, 15 % masked (max_predictions 20 @128 / 80 @512
    as in the NVIDIA/Google pretraining recipe), AdamW, dropout 0.1 on."""
    V = 30522
    S = a.seq
    P = max(1, round(0.15 * S)) if S != 128 else 20
    R = a.emulate_ranks
    if R > 1 and (world != 1 or a.impl != "mipipe"):
        raise SystemExit("--emulate-ranks is a world-1 mipipe reference run")

    def rank_batches(r):
        g = torch.Generator(device=dev)
        g.manual_seed(1234 + r)
        out = []
        for _ in range(2):
            ids = torch.randint(0, V, (a.batch, S), device=dev, generator=g)
            am = torch.ones(a.batch, S, device=dev, dtype=torch.int64)
            pos = torch.stack([torch.randperm(S, device=dev, generator=g)[:P]
                               for _ in range(a.batch)])
            labels = torch.randint(0, V, (a.batch, P), device=dev, generator=g)
            out.append((ids, am, pos, labels))
        return out

    if R > 1:
        # step batch i = the R per-rank batches ranks 0..R-1 would each draw for their step i
        per = [rank_batches(r) for r in range(R)]
        batches = [tuple(torch.cat([per[r][i][k] for r in range(R)]) for k in range(4))
                   for i in range(2)]
    else:
        batches = rank_batches(rank)
    if a.impl == "mipipe":
        from mipipe.models import create_model
        from mipipe.optim import AdamW
        from mipipe.parallel import DistributedDataParallel
        drop = {} if a.bert_dropout is None else {
            "hidden_dropout_prob": a.bert_dropout, "attention_probs_dropout_prob": a.bert_dropout}
        model = create_model(a.model, **drop).to(dev)
        model.compute_dtype = _compute_dtype(a)
        if a.distributed:
            model = DistributedDataParallel(model, device_ids=[local], bucket_cap_mb=a.bucket_cap_mb,
                                            force_reduce=a.force_reduce,
                                            comm_dtype=_comm_dtype(a))
        opt = AdamW(model.parameters(), lr=1e-4, weight_decay=0.01)

        def step(ids, am, pos, labels):
            opt.zero_grad()
            loss = model(ids, am, masked_positions=pos, labels=labels)
            loss.backward()
            opt.step()
            return loss

        if R > 1:
            def step(ids, am, pos, labels):  # noqa: F811
                # one forward / backward per emulated rank (its own dropout seeds: the rank's
                # seed offset at the step counter every rank would be at), loss / R each: the
                # mean of per-rank gradients that DDP's averaged all-reduce produces
                opt.zero_grad()
                s0 = model._step
                sd0 = model._step_dev.clone() if model._step_dev is not None else None
                total = 0.0
                chunks = [t.chunk(R) for t in (ids, am, pos, labels)]
                for r in range(R):
                    model.rank_override = r
                    model._step = s0
                    if sd0 is not None:
                        model._step_dev.copy_(sd0)
                    loss = model(chunks[0][r], chunks[1][r], masked_positions=chunks[2][r],
                                 labels=chunks[3][r]) / R
                    loss.backward()
                    total = total + loss.detach()
                model.rank_override = None
                opt.step()
                return total

        # AdamW's step count and the dropout seeds' per-step part live on the device, so the
        # whole step (dropout included) replays from one captured hipGraph
        from mipipe.train.graph import GraphedStep, graph_safe
        ok, why = graph_safe(model, opt)
        if dev.type == "cpu":
            ok, why = False, "no hipGraph on the CPU"
        if R > 1:
            ok, why = False, "--emulate-ranks runs eagerly"
        if a.graph == "on" or (a.graph == "auto" and ok):
            if not ok:
                raise SystemExit(f"--graph on is not possible here: {why}")
            model.train()
            gs = _capture(GraphedStep, step, batches, a)
            if gs is not None:
                ids_of = {id(b[0]): k for k, b in enumerate(batches)}

                def step(ids, am, pos, labels):  # noqa: F811
                    return gs.replay(ids_of[id(ids)])
    else:
        from mipipe.models.reference import ref_bert
        model = ref_bert(a.model).to(dev)
        if world > 1:
            model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local])
        opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01, fused=True)
        inner = model.module if world > 1 else model

        def step(ids, am, pos, labels):
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits = model(ids, am, masked_positions=pos)
            loss = inner.loss(logits, labels)
            loss.backward()
            opt.step()
            return loss
    return step, model, batches


def _capture(GraphedStep, step, batches, a):
    """Capture the step into hipGraphs; with ``--graph auto`` a CAPTURE that fails on any rank
    makes every rank run eagerly (one MIN all-reduce of a success flag after the attempt —
    captured collectives never execute during capture, so a rank whose capture failed cannot
    leave peers waiting inside one).  A failure in GraphedStep's eager warm-up steps (real DDP
    collectives) is not caught: that rank exits non-zero and the launcher's fail-fast ends the
    job, instead of a MIN all-reduce that would pair with its peers' bucket collectives.
    ``--graph on`` re-raises."""
    import torch.distributed as dist
    from mipipe.train.graph import CaptureFailed
    gs, err = None, None
    try:
        gs = GraphedStep(step, batches[0], warmup=max(2, a.warmup), inputs=batches)
    except CaptureFailed as exc:  # reported, then handled uniformly across ranks
        err = exc
        if a.graph == "on":
            raise
    ok = torch.tensor([0 if err is not None else 1], dtype=torch.int32,
                      device=batches[0][0].device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) == 0:
        torch.cuda.synchronize()
        print(f"[bench] hipGraph capture failed ({err!r} on this rank or a peer); running the "
              "step eagerly", file=sys.stderr, flush=True)
        a.graph_used = False
        return None
    a.graph_used = True
    return gs


def _rccl_settings():
    from mipipe.parallel.dist_utils import rccl_settings
    return rccl_settings()


def _comm_dtype(a):
    return torch.bfloat16 if a.comm_dtype == "bf16" else None


def _compute_dtype(a):
    return torch.float32 if (a.device == "cpu" or a.dtype == "fp32") else torch.bfloat16


def build_cnn(a, world, local, dev, rank):
    from mipipe.data.synthetic import synthetic_batch
    idx = [torch.arange(i * a.batch, (i + 1) * a.batch, device=dev) + rank * 10_000_000
           for i in range(2)]
    in_ch = 1 if a.model == "mnist_cnn" else 3
    batches = [synthetic_batch(t, (in_ch, a.res, a.res), a.classes, seed=0) for t in idx]
    R = a.emulate_ranks
    if R > 1:
        if world != 1 or a.impl != "mipipe":
            raise SystemExit("--emulate-ranks is a world-1 mipipe reference run")
        # step batch i = the R chunks ranks 0..R-1 would each draw for their step i
        batches = []
        for i in range(2):
            parts = [synthetic_batch(torch.arange(i * a.batch, (i + 1) * a.batch, device=dev)
                                     + r * 10_000_000, (in_ch, a.res, a.res), a.classes, seed=0)
                     for r in range(R)]
            batches.append((torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts])))

    if a.impl == "mipipe":
        from mipipe.models import create_model
        from mipipe.optim import SGD
        from mipipe.parallel import DistributedDataParallel
        from mipipe.train.task import CrossEntropyLoss
        cross_entropy = CrossEntropyLoss()  # also sums GoogLeNet / Inception-v3 aux losses
        model = create_model(a.model, num_classes=a.classes).to(dev)
        model.compute_dtype = _compute_dtype(a)
        if a.distributed:
            model = DistributedDataParallel(model, device_ids=[local], bucket_cap_mb=a.bucket_cap_mb,
                                            force_reduce=a.force_reduce,
                                            comm_dtype=_comm_dtype(a))
        # fp32 compute reads the fp32 master weights directly: no bf16 shadow to refresh
        opt = SGD(model.parameters(), 0.1, momentum=0.9, weight_decay=1e-4,
                  shadow_dtype=None if _compute_dtype(a) == torch.float32 else "auto")

        def step(x, y):
            opt.zero_grad()
            loss = cross_entropy(model(x), y)
            loss.backward()
            opt.step()
            return loss

        if R > 1:
            def step(x, y):  # noqa: F811
                opt.zero_grad()
                bufs = list(model.buffers())
                start = [b.detach().clone() for b in bufs]  # rank 0's broadcast buffers
                after0, total = None, 0.0
                for r, (xr, yr) in enumerate(zip(x.chunk(R), y.chunk(R))):
                    for b, s0 in zip(bufs, start):
                        b.copy_(s0)
                    loss = cross_entropy(model(xr), yr) / R  # DDP: mean of per-rank gradients
                    loss.backward()
                    if r == 0:
                        after0 = [b.detach().clone() for b in bufs]
                    total = total + loss.detach()
                for b, s1 in zip(bufs, after0):
                    b.copy_(s1)
                opt.step()
                return total

        from mipipe.train.graph import GraphedStep, graph_safe
        ok, why = graph_safe(model, opt)
        if dev.type == "cpu":
            ok, why = False, "no hipGraph on the CPU"
        if R > 1:
            ok, why = False, "--emulate-ranks runs eagerly"
        if a.graph == "on" or (a.graph == "auto" and ok):
            if not ok:
                raise SystemExit(f"--graph on is not possible here: {why}")
            model.train()
            # one captured step per resident synthetic batch: replays issue every kernel of the
            # step (fwd, bwd, SGD) from one launch; no batch copies
            gs = _capture(GraphedStep, step, batches, a)
            if gs is not None:
                ids = {id(b[0]): k for k, b in enumerate(batches)}

                def step(x, y):  # noqa: F811
                    return gs.replay(ids[id(x)])
    else:
        from mipipe.models.reference import _RESNET_CFG, ref_resnet
        if a.model in _RESNET_CFG:
            model = ref_resnet(a.model, num_classes=a.classes)
            call = model
        else:
            # torchvision-structured zoo model: its plain-torch module tree (MIOpen convs/BN,
            # ATen elementwise) is exactly stock PyTorch-ROCm running that architecture
            from mipipe.models import create_model
            if world > 1:
                raise SystemExit("--impl stock: zoo models are benchmarked on one GPU")
            model = create_model(a.model, num_classes=a.classes)
            call = model.reference_forward
        # channels_last for the ResNets (MIOpen's fastest layout there, as measured for
        # BASELINE.md); default NCHW for the zoo (MIOpen's NHWC depthwise / grouped convs are
        # several times slower than its NCHW ones)
        cl = a.model in _RESNET_CFG
        model = model.to(dev).to(memory_format=torch.channels_last if cl else torch.contiguous_format)
        if world > 1:
            model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local])
            call = model
        opt = torch.optim.SGD(model.parameters(), 0.1, momentum=0.9, weight_decay=1e-4)
        # MIOpen benchmark-mode search for ResNets (as measured for BASELINE.md); the zoo's many
        # depthwise / grouped shapes use MIOpen's immediate mode (the search takes minutes)
        torch.backends.cudnn.benchmark = a.model in _RESNET_CFG
        if cl:
            batches = [(x.contiguous(memory_format=torch.channels_last), y) for x, y in batches]

        def crit(out, y):
            f = torch.nn.functional.cross_entropy
            if isinstance(out, tuple):  # aux heads, weighted like mipipe's CrossEntropyLoss
                w = 0.4 if len(out) == 2 else 0.3
                return f(out[0], y) + sum(w * f(o, y) for o in out[1:] if o is not None)
            return f(out, y)

        amp = a.dtype == "bf16" and dev.type == "cuda"

        def step(x, y):
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                loss = crit(call(x), y)
            loss.backward()
            opt.step()
            return loss

    return step, model, batches


if __name__ == "__main__":
    sys.exit(main())
