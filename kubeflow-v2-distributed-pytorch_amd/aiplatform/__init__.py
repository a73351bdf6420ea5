"""Training-job API (replaces ``google.cloud.aiplatform`` for the reference's ``train`` step).

Reference (pytorch-pipeline.ipynb nb:134-196)::

    aiplatform.init(project=PROJECT_ID, location=REGION, staging_bucket=BUCKET_NAME)
    job = aiplatform.CustomTrainingJob(display_name=JOB_NAME, script_path=input_file_path,
                                       container_uri=TRAIN_IMAGE, staging_bucket=base_output_dir)
    model = job.run(args=ARGS, replica_count=3, machine_type="n1-standard-16",
                    accelerator_type="NVIDIA_TESLA_V100", accelerator_count=2)

Here ``run`` stages the script into the local object store, then starts
``replica_count`` processes on this node through :mod:`mipipe.launch`, each pinned to
``accelerator_count`` MI355X GPUs, with Vertex's env contract (``WORLD_SIZE``, ``RANK``,
``MASTER_ADDR/PORT``, ``AIP_MODEL_DIR``, ``CLUSTER_SPEC``).  ``container_uri`` and
``machine_type`` are recorded but there are no containers/VMs: the job runs in this
image's Python.  Any ``accelerator_type`` other than ``AMD_INSTINCT_MI355X`` is accepted and
mapped onto the node's MI355X GPUs (the reference asked for V100s).
"""
from __future__ import annotations

import datetime as _dt
import enum
import json
import os
import shutil
import sys
import types
from typing import Any, Dict, List, Optional, Sequence

from mipipe.launch.launcher import LaunchSpec, launch
from mipipe.storage.gcs import uri_to_local_path

__all__ = ["init", "CustomTrainingJob", "CustomJob", "Model", "gapic", "JobFailed"]

_config: Dict[str, Any] = {"project": "local", "location": "local", "staging_bucket": None}


def init(project: Optional[str] = None, location: Optional[str] = None,
         staging_bucket: Optional[str] = None, experiment: Optional[str] = None,
         credentials=None, **_: Any) -> None:
    if project:
        _config["project"] = project
    if location:
        _config["location"] = location
    if staging_bucket:
        _config["staging_bucket"] = staging_bucket
    if experiment:
        _config["experiment"] = experiment


class AcceleratorType(enum.Enum):
    ACCELERATOR_TYPE_UNSPECIFIED = 0
    NVIDIA_TESLA_K80 = 1
    NVIDIA_TESLA_P100 = 2
    NVIDIA_TESLA_V100 = 3
    NVIDIA_TESLA_P4 = 4
    NVIDIA_TESLA_T4 = 5
    NVIDIA_TESLA_A100 = 8
    AMD_INSTINCT_MI355X = 100


gapic = types.SimpleNamespace(AcceleratorType=AcceleratorType)


class JobFailed(RuntimeError):
    pass


class Model:
    """Handle to the model directory a job exported (``AIP_MODEL_DIR``)."""

    def __init__(self, display_name: str, artifact_uri: str):
        self.display_name = display_name
        self.uri = artifact_uri
        self.resource_name = f"projects/{_config['project']}/locations/{_config['location']}/models/{display_name}"

    @property
    def local_path(self) -> str:
        return uri_to_local_path(self.uri)

    def __repr__(self) -> str:
        return f"aiplatform.Model({self.display_name!r}, uri={self.uri!r})"


def _ts() -> str:
    return _dt.datetime.now().strftime("%Y%m%d%H%M%S")


def _accel_name(a) -> Optional[str]:
    if a is None:
        return None
    if isinstance(a, AcceleratorType):
        return a.name
    return str(a)


class CustomTrainingJob:
    def __init__(self, display_name: str, script_path: str, container_uri: Optional[str] = None,
                 requirements: Optional[Sequence[str]] = None,
                 model_serving_container_image_uri: Optional[str] = None,
                 staging_bucket: Optional[str] = None, project: Optional[str] = None,
                 location: Optional[str] = None, **_: Any):
        self.display_name = display_name
        self.script_path = uri_to_local_path(script_path)
        self.container_uri = container_uri
        self.requirements = list(requirements or [])
        self.staging_bucket = staging_bucket or _config.get("staging_bucket") or "gs://mipipe-staging"
        self.state = "JOB_STATE_QUEUED"
        self.resource_name = f"projects/{project or _config['project']}/locations/" \
                             f"{location or _config['location']}/trainingPipelines/{display_name}"
        self.last_launch: Optional[LaunchSpec] = None

    def _stage_script(self, job_dir: str) -> str:
        """Package the script like Vertex's source distribution: copy it into
        ``<staging>/<job>/`` and run it from there."""
        if not os.path.isfile(self.script_path):
            raise FileNotFoundError(f"training script not found: {self.script_path}")
        staged_dir = uri_to_local_path(f"{job_dir}/code")
        os.makedirs(staged_dir, exist_ok=True)
        name = os.path.basename(self.script_path)
        if not name.endswith(".py"):
            name = "task.py"
        dst = os.path.join(staged_dir, name)
        shutil.copyfile(self.script_path, dst)
        return dst

    def run(self, args: Optional[List[str]] = None, replica_count: int = 1,
            machine_type: str = "local", accelerator_type=None, accelerator_count: int = 0,
            base_output_dir: Optional[str] = None, model_display_name: Optional[str] = None,
            environment_variables: Optional[Dict[str, str]] = None, sync: bool = True,
            timeout: Optional[float] = None, nproc_per_node: Optional[int] = None,
            gpu_visibility: str = "auto", **_: Any) -> Optional[Model]:
        """``gpu_visibility`` (mipipe extension, launch/env.py): "slice" = each replica sees
        only its ``accelerator_count`` GPUs (a Vertex VM; default when replicas share the
        node), "all" = every GPU visible, slice named by MIPIPE_DEVICE_OFFSET (xGMI P2P across
        replicas; for mipipe-aware scripts)."""
        if replica_count < 1:
            raise ValueError("replica_count must be >= 1")
        base = (base_output_dir or f"{self.staging_bucket.rstrip('/')}/"
                f"aiplatform-custom-training-{_ts()}").rstrip("/")
        script = self._stage_script(base)
        model_dir = f"{base}/model/"
        os.makedirs(uri_to_local_path(model_dir), exist_ok=True)
        accel = _accel_name(accelerator_type)
        env = dict(environment_variables or {})
        env.setdefault("AIP_TRAINING_DATA_URI", "")
        env["MIPIPE_ACCELERATOR_TYPE"] = accel or "NONE"
        env["MIPIPE_MACHINE_TYPE"] = machine_type
        repo_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = repo_root + (os.pathsep + os.environ["PYTHONPATH"]
                                         if os.environ.get("PYTHONPATH") else "")
        spec = LaunchSpec(command=[sys.executable, script] + list(args or []),
                          replica_count=replica_count,
                          accelerator_count=accelerator_count if accel else 0,
                          nproc_per_node=nproc_per_node, env=env, model_dir=model_dir,
                          checkpoint_dir=f"{base}/checkpoints/",
                          tensorboard_dir=f"{base}/logs/",
                          log_dir=uri_to_local_path(f"{base}/logs"), timeout=timeout,
                          cwd=os.path.dirname(script), gpu_visibility=gpu_visibility)
        self.last_launch = spec
        record = {"displayName": self.display_name, "containerUri": self.container_uri,
                  "machineType": machine_type, "acceleratorType": accel,
                  "acceleratorCount": accelerator_count, "replicaCount": replica_count,
                  "args": list(args or []), "baseOutputDirectory": base}
        with open(os.path.join(uri_to_local_path(base), "job.json"), "w") as f:
            json.dump(record, f, indent=2)
        self.state = "JOB_STATE_RUNNING"
        rc = launch(spec)
        self.state = "JOB_STATE_SUCCEEDED" if rc == 0 else "JOB_STATE_FAILED"
        if rc != 0:
            raise JobFailed(f"training job {self.display_name} failed with exit code {rc}; "
                            f"logs in {spec.log_dir}")
        if model_display_name:
            return Model(model_display_name, model_dir)
        return None


class CustomJob:
    """``worker_pool_specs`` form: one pool spec per replica group (first is the chief)."""

    def __init__(self, display_name: str, worker_pool_specs: List[Dict[str, Any]],
                 base_output_dir: Optional[str] = None, staging_bucket: Optional[str] = None,
                 **_: Any):
        self.display_name = display_name
        self.pools = worker_pool_specs
        self.base_output_dir = base_output_dir
        self.staging_bucket = staging_bucket or _config.get("staging_bucket") or "gs://mipipe-staging"

    def run(self, sync: bool = True, timeout: Optional[float] = None, **_: Any) -> None:
        replicas = sum(int(p.get("replica_count", 1)) for p in self.pools)
        first = self.pools[0]
        spec = first.get("python_package_spec") or first.get("container_spec") or {}
        script = spec.get("script_path") or spec.get("python_module") or spec.get("command", [None])[0]
        args = spec.get("args", [])
        ms = first.get("machine_spec", {})
        job = CustomTrainingJob(self.display_name, script, staging_bucket=self.staging_bucket)
        job.run(args=args, replica_count=replicas, accelerator_type=ms.get("accelerator_type"),
                accelerator_count=int(ms.get("accelerator_count", 0)),
                base_output_dir=self.base_output_dir, timeout=timeout)
