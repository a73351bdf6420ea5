"""BASELINE config 5: a 3-step kfp.v2 pipeline  preprocess -> train -> eval (+ gated deploy).

The reference pipeline declares ``baseline_accuracy`` but never uses it (SURVEY.md §2.1 O6,
pytorch-pipeline.ipynb:218-221); its notebook placeholders (nb:10, nb:20) ask for a data step
before training.  This pipeline completes that design on one MI355X node:

1. ``preprocess`` writes the dataset as CIFAR-binary record files (synthetic & learnable: no
   network) into a ``Dataset`` artifact;
2. ``train`` launches the distributed training job through the aiplatform-compatible job API
   (local launcher, one rank per GPU, RCCL DDP) running mipipe's task.py on those records via
   the native multi-threaded loader; the trained model lands in a ``Model`` artifact;
3. ``evaluate`` scores the model on the test records (HIP kernels on GPU), logs accuracy and a
   confusion matrix, and decides ``deploy`` against ``baseline_accuracy``;
4. ``deploy`` (inside ``dsl.Condition(deploy == "true")``) publishes the model to the serving
   directory.

Run (8 GPUs, ResNet-50 @ CIFAR shape):
  python examples/three_step_pipeline.py --gpus 8 --arch resnet50 --epochs 2
CPU smoke (config 1 style):
  python examples/three_step_pipeline.py --gpus 0 --arch mnist_cnn --dataset mnist --epochs 1
"""
import argparse
import json
import os
import sys
from typing import NamedTuple

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mipipe import kfp  # noqa: E402
from mipipe.dsl import (component, Input, Output, Dataset, Model, Metrics,  # noqa: E402
                        ClassificationMetrics)


@component()
def preprocess(dataset: str, n_train: int, n_test: int, seed: int, data: Output[Dataset]):
    import json
    import os
    from mipipe.data.records import write_synthetic_dataset
    man = write_synthetic_dataset(data.path, dataset, n_train=n_train, n_test=n_test, seed=seed)
    data.metadata.update({k: v for k, v in man.items() if k != "files"})
    with open(os.path.join(data.path, "manifest.json"), "w") as f:
        json.dump(man, f)
    print(f"wrote {n_train}+{n_test} {dataset} records to {data.path}")


@component()
def train(data: Input[Dataset], arch: str, dataset: str, epochs: int, batch_size: int,
          gpus: int, learning_rate: float, extra_args: str, model: Output[Model],
          metrics: Output[Metrics]) -> float:
    import json
    import os
    from datetime import datetime
    from google.cloud import aiplatform
    from google.cloud.aiplatform import gapic as aip
    import mipipe.train.task as task_mod

    ts = datetime.now().strftime("%Y_%m_%d_%H_%M_%S")
    aiplatform.init(project="local", location="local")
    args = ["--dist-url=env://", f"--arch={arch}", f"--dataset={dataset}",
            f"--data-dir={data.path}", f"--num_epochs={epochs}", f"--batch_size={batch_size}",
            f"--learning_rate={learning_rate}", "--eval-every=1000", "--log-every=10",
            "--model_filename=model.pth", f"--num_classes={int(data.metadata.get('num_classes', 10))}"
            ] + json.loads(extra_args)
    if gpus > 1:
        args.append("--multiprocessing-distributed")
    job = aiplatform.CustomTrainingJob(display_name=f"train_{arch}_{ts}",
                                       script_path=task_mod.__file__, container_uri="local")
    accel = aip.AcceleratorType.AMD_INSTINCT_MI355X if gpus else None
    job.run(args=args, replica_count=1, machine_type="local",
            accelerator_type=accel.name if accel else None, accelerator_count=gpus,
            base_output_dir=model.path)
    acc, found = 0.0, False
    for root, _, files in os.walk(model.path):
        for fn in files:
            if fn.endswith(".log"):
                with open(os.path.join(root, fn)) as f:
                    for line in f:
                        if "MIPIPE_METRICS" in line:
                            m = json.loads(line.split("MIPIPE_METRICS", 1)[1])
                            found = True
                            acc = float(m["accuracy"])
                            for k, v in m.items():
                                if isinstance(v, (int, float)):
                                    metrics.log_metric(k, v)
    if not found:
        raise RuntimeError("training job produced no metrics line")
    model.metadata.update({"arch": arch, "dataset": dataset, "framework": "mipipe"})
    return acc * 100.0


@component()
def evaluate(data: Input[Dataset], model: Input[Model], arch: str, dataset: str,
             baseline_accuracy: float, metrics: Output[ClassificationMetrics],
             summary: Output[Metrics]) -> NamedTuple("EvalOutput", [("accuracy", float),
                                                                     ("deploy", str)]):
    import os
    from collections import namedtuple
    import torch
    from mipipe.data import records as REC
    from mipipe.models import create_model
    from mipipe.train.checkpoint import strip_module_prefix

    path = None
    for root, _, files in os.walk(model.path):
        for fn in files:
            if fn == "model.pth":
                path = os.path.join(root, fn)
    if path is None:
        raise FileNotFoundError(f"no model.pth under {model.path}")
    shape = (3, 32, 32) if dataset == "cifar10" else (1, 28, 28)
    sd = strip_module_prefix(torch.load(path, map_location="cpu", weights_only=True))
    head = [v for k, v in sd.items() if v.dim() == 2][-1]  # classifier weight [classes, feat]
    ncls = int(head.shape[0])
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    net = create_model(arch, num_classes=ncls)
    net.load_state_dict(sd)
    net = net.to(dev).eval()
    mean, std = ((REC.MNIST_MEAN, REC.MNIST_STD) if dataset == "mnist"
                 else (REC.CIFAR10_MEAN, REC.CIFAR10_STD))
    files = REC.dataset_files(data.path, dataset, "test")
    loader = REC.RecordDataLoader(files, shape, 256, train=False, mean=mean, std=std,
                                  device=dev)
    cm = torch.zeros(ncls, ncls, dtype=torch.int64, device=dev)
    with torch.no_grad():
        for x, y in loader:
            pred = net(x).float().argmax(1)
            cm.index_put_((y, pred), torch.ones_like(y), accumulate=True)
    cm = cm.cpu()
    acc = 100.0 * float(cm.diag().sum()) / max(1, int(cm.sum()))
    cats = [str(i) for i in range(ncls)]
    metrics.log_confusion_matrix(cats, cm.tolist())
    summary.log_metric("accuracy", acc)
    summary.log_metric("baseline_accuracy", baseline_accuracy)
    deploy = "true" if acc >= baseline_accuracy else "false"
    summary.log_metric("deploy", 1.0 if deploy == "true" else 0.0)
    print(f"test accuracy {acc:.2f}% vs baseline {baseline_accuracy}% -> deploy={deploy}")
    out = namedtuple("EvalOutput", ["accuracy", "deploy"])
    return out(acc, deploy)


@component()
def deploy(model: Input[Model], serving_dir: str) -> str:
    import os
    import shutil
    dst = os.path.join(serving_dir, os.path.basename(model.path.rstrip("/")))
    shutil.copytree(model.path, dst, dirs_exist_ok=True)
    print(f"deployed {model.path} -> {dst}")
    return dst


@kfp.dsl.pipeline(name="preprocess-train-eval")
def pipeline(baseline_accuracy: float = 70.0, dataset: str = "cifar10", arch: str = "resnet50",
             n_train: int = 10000, n_test: int = 2000, epochs: int = 2, batch_size: int = 256,
             gpus: int = 8, learning_rate: float = 0.1, extra_args: str = "[]",
             serving_dir: str = "/tmp/mipipe_serving", seed: int = 0):
    pre = preprocess(dataset, n_train, n_test, seed)
    tr = train(pre.outputs["data"], arch, dataset, epochs, batch_size, gpus, learning_rate,
               extra_args)
    ev = evaluate(pre.outputs["data"], tr.outputs["model"], arch, dataset, baseline_accuracy)
    with kfp.dsl.Condition(ev.outputs["deploy"] == "true"):
        deploy(tr.outputs["model"], serving_dir)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--dataset", default="cifar10")
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--n-train", type=int, default=10000)
    ap.add_argument("--n-test", type=int, default=2000)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--baseline-accuracy", type=float, default=70.0)
    ap.add_argument("--extra-args", default="[]")
    ap.add_argument("--serving-dir", default="/tmp/mipipe_serving")
    ap.add_argument("--spec", default="three_step.json")
    ap.add_argument("--pipeline-root", default="gs://mipipe/pipeline_root")
    a = ap.parse_args(argv)
    from mipipe.kfp.v2 import compiler
    from mipipe.kfp.v2.google.client import AIPlatformClient
    compiler.Compiler().compile(pipeline_func=pipeline, package_path=a.spec)
    client = AIPlatformClient(project_id="local", region="local")
    resp = client.create_run_from_job_spec(
        a.spec, pipeline_root=a.pipeline_root,
        parameter_values={"baseline_accuracy": a.baseline_accuracy, "dataset": a.dataset,
                          "arch": a.arch, "n_train": a.n_train, "n_test": a.n_test,
                          "epochs": a.epochs, "batch_size": a.batch_size, "gpus": a.gpus,
                          "learning_rate": a.lr, "extra_args": a.extra_args,
                          "serving_dir": a.serving_dir}, sync=True)
    run = client.get_run(resp["runId"])
    print(json.dumps({"run": resp["runId"], "state": run["state"],
                      "tasks": {k: v.get("state") for k, v in run.get("tasks", {}).items()}}))
    return 0 if run["state"] == "PIPELINE_STATE_SUCCEEDED" else 1


if __name__ == "__main__":
    sys.exit(main())
