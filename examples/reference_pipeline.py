"""The reference notebook's pipeline (pytorch-pipeline.ipynb cells 5-11), on mipipe.

Same two components and wiring: ``download_file(bucket, blob) -> output_file`` then
``train(input_file)``, where ``train`` launches a multi-replica training job running the
downloaded ``task.py`` through the aiplatform-compatible job API.  Differences from the
reference, all forced by running on one offline MI355X node:
  * the object store is local (``gs://`` -> $MIPIPE_GCS_ROOT), so the component bodies stay
    byte-for-byte the reference's GCS calls;
  * the training job's topology is a component parameter (replicas x GPUs per replica)
    instead of hard-coded V100 VMs; ``accelerator_count=0`` runs on CPU/gloo (config 1).

Run:  python examples/reference_pipeline.py --replicas 1 --gpus-per-replica 0
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mipipe import kfp  # noqa: E402  (kfp-compatible import surface)
from mipipe.dsl import component, InputPath, OutputPath, Output, Metrics  # noqa: E402


@component(packages_to_install=["google-cloud-storage"])
def download_file(bucket_name: str, source_blob_name: str, output_file_path: OutputPath()):
    from google.cloud import storage
    storage_client = storage.Client()
    bucket = storage_client.bucket(bucket_name)
    blob = bucket.blob(source_blob_name)
    blob.download_to_filename(output_file_path)
    print("Downloaded storage object {} from bucket {} to local file {}.".format(
        source_blob_name, bucket_name, output_file_path))


@component(packages_to_install=["google-cloud-aiplatform", "google-cloud-storage"])
def train(input_file_path: InputPath(), metrics: Output[Metrics], replica_count: int = 1,
          accelerator_count: int = 0, num_epochs: int = 2, extra_args: str = "[]") -> float:
    import json
    import os
    from datetime import datetime
    from google.cloud import aiplatform
    from google.cloud.aiplatform import gapic as aip

    aiplatform.init(project="local", location="local", staging_bucket="gs://test-pkl")
    TIMESTAMP = datetime.now().strftime("%Y_%m_%d_%H_%M_%S")
    JOB_NAME = "cifar10_resnet_custom_job_" + TIMESTAMP
    ARGS = ["--dist-url=env://", "--multiprocessing-distributed",
            f"--num_epochs={num_epochs}"] + json.loads(extra_args)
    base_output_dir = "gs://test-pkl/jobs/{}".format(JOB_NAME)
    job = aiplatform.CustomTrainingJob(display_name=JOB_NAME, script_path=input_file_path,
                                       container_uri="local", staging_bucket=base_output_dir)
    accel = aip.AcceleratorType.AMD_INSTINCT_MI355X if accelerator_count else None
    model = job.run(args=ARGS, replica_count=replica_count, machine_type="local",
                    accelerator_type=accel.name if accel else None,
                    accelerator_count=accelerator_count, base_output_dir=base_output_dir,
                    model_display_name="cifar10-pytorch-" + TIMESTAMP)
    # task.py prints a MIPIPE_METRICS line on rank 0; the launcher keeps per-rank logs
    from mipipe.storage.gcs import uri_to_local_path
    acc = 0.0
    log = os.path.join(uri_to_local_path(base_output_dir), "logs", "rank0.log")
    with open(log) as f:
        for line in f:
            if "MIPIPE_METRICS" in line:
                m = json.loads(line.split("MIPIPE_METRICS", 1)[1])
                acc = float(m["accuracy"])
                for k, v in m.items():
                    if isinstance(v, (int, float)):
                        metrics.log_metric(k, v)
    metrics.metadata["model_uri"] = model.uri
    return acc * 100.0


@kfp.dsl.pipeline(name="download-file-local")
def pipeline(baseline_accuracy: float = 70.0, replica_count: int = 1, accelerator_count: int = 0,
             num_epochs: int = 2, extra_args: str = "[]"):
    download_file_task = download_file("test-pkl", "task.py")
    train(download_file_task.output, replica_count=replica_count,
          accelerator_count=accelerator_count, num_epochs=num_epochs, extra_args=extra_args)


def stage_task_script(bucket: str = "test-pkl", name: str = "task.py") -> str:
    """Upload mipipe's task.py into the local object store (what the reference did by hand)."""
    from mipipe.storage import gcs
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "kubeflow-v2-distributed-pytorch_amd", "train", "task.py")
    gcs.Client().bucket(bucket).blob(name).upload_from_filename(src)
    return f"gs://{bucket}/{name}"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=1)
    ap.add_argument("--gpus-per-replica", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--extra-args", default=json.dumps(
        ["--arch=mnist_cnn", "--dataset=mnist", "--batch_size=64", "--train-samples=512",
         "--test-samples=256", "--eval-every=1"]))
    ap.add_argument("--spec", default="dag.json")
    ap.add_argument("--env-file", default=".env", help="PROJECT_ID / BUCKET (notebook nb:73-86)")
    a = ap.parse_args(argv)
    from mipipe.kfp.v2 import compiler
    from mipipe.kfp.v2.google.client import AIPlatformClient
    from mipipe.utils import load_dotenv, pipeline_config
    load_dotenv(a.env_file)  # the notebook's `%load_ext dotenv` + `%dotenv`
    cfg = pipeline_config()
    stage_task_script()
    compiler.Compiler().compile(pipeline_func=pipeline, package_path=a.spec)
    client = AIPlatformClient(project_id=cfg.project_id, region=cfg.region)
    resp = client.create_run_from_job_spec(
        a.spec, pipeline_root=cfg.pipeline_root,
        parameter_values={"baseline_accuracy": 80.0, "replica_count": a.replicas,
                          "accelerator_count": a.gpus_per_replica, "num_epochs": a.epochs,
                          "extra_args": a.extra_args}, sync=True)
    run = client.get_run(resp["runId"])
    print(json.dumps({"run": resp["runId"], "state": run["state"]}))
    return 0 if run["state"] == "PIPELINE_STATE_SUCCEEDED" else 1


if __name__ == "__main__":
    sys.exit(main())
