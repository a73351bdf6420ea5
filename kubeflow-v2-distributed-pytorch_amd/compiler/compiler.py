"""DSL -> kfp v2 pipeline-spec JSON compiler.

Reference: ``compiler.Compiler().compile(pipeline_func=pipeline,
package_path="dag-"+TIMESTAMP+".json")`` (pytorch-pipeline.ipynb nb:231-234).  The
emitted document is the kfp 1.8 "v2" job spec: ``{"pipelineSpec": {
pipelineInfo, root{dag, inputDefinitions}, components{comp-*}, deploymentSpec{executors
{exec-*}}, schemaVersion "2.0.0", sdkVersion}, "runtimeConfig": {parameters}}``.
kfp itself is not installed (no network), so the schema is pinned by golden tests
(tests/test_compiler.py) instead of a round-trip through kfp.
"""
from __future__ import annotations

import inspect
import json
from typing import Any, Dict, List, Optional, Tuple

from mipipe import __version__
from mipipe.dsl.component import Component
from mipipe.dsl.pipeline import (ConditionOperator, Pipeline, PipelineBuilder, PipelineParam,
                                 PipelineTask, TaskOutput, _Group)

SCHEMA_VERSION = "2.0.0"
SDK_VERSION = f"mipipe-{__version__}"
ARTIFACT_SCHEMA_VERSION = "0.0.1"

__all__ = ["Compiler", "compile_pipeline", "component_to_yaml", "SCHEMA_VERSION"]


def _constant_value(v: Any, ptype: str) -> Dict[str, Any]:
    if ptype == "INT":
        return {"intValue": str(int(v))}
    if ptype == "DOUBLE":
        return {"doubleValue": float(v)}
    if isinstance(v, (dict, list, bool)):
        return {"stringValue": json.dumps(v)}
    return {"stringValue": str(v)}


def _value_accessor(ptype: str) -> str:
    return {"INT": "int_value", "DOUBLE": "double_value"}.get(ptype, "string_value")


def _channel_type(ch) -> Tuple[str, str]:
    """(kind, type) for a channel."""
    if isinstance(ch, PipelineParam):
        return "parameter", ch.param_type
    if isinstance(ch, TaskOutput):
        return ch.kind, ch.type
    raise TypeError(ch)


def _external_name(ch) -> str:
    if isinstance(ch, PipelineParam):
        return f"pipelineparam--{ch.name}"
    return f"pipelineparam--{ch.task.name}-{ch.name}"


class _Ctx:
    def __init__(self, builder: PipelineBuilder):
        self.builder = builder
        self.components: Dict[str, Any] = {}
        self.executors: Dict[str, Any] = {}
        self._comp_names: Dict[int, str] = {}
        self._used_names: Dict[str, int] = {}

    def component_name(self, comp: Component) -> str:
        key = id(comp)
        if key in self._comp_names:
            return self._comp_names[key]
        base = f"comp-{comp.name}"
        n = self._used_names.get(base, 0) + 1
        self._used_names[base] = n
        name = base if n == 1 else f"{base}-{n}"
        self._comp_names[key] = name
        exec_label = "exec-" + name[len("comp-"):]
        self.components[name] = self._component_spec(comp, exec_label)
        if getattr(comp, "is_importer", False):
            self.executors[exec_label] = {"importer": {
                "artifactUri": {"runtimeParameter": "uri"},
                "typeSchema": comp.importer_spec["typeSchema"],
                "reimport": comp.importer_spec["reimport"],
                "metadata": comp.importer_spec["metadata"]}}
        else:
            self.executors[exec_label] = {"container": comp.container_spec()}
        return name

    @staticmethod
    def _component_spec(comp: Component, exec_label: str) -> Dict[str, Any]:
        spec: Dict[str, Any] = {"executorLabel": exec_label}
        ind: Dict[str, Any] = {}
        for s in comp.inputs:
            if s.kind == "parameter":
                ind.setdefault("parameters", {})[s.name] = {"type": s.type}
            else:
                ind.setdefault("artifacts", {})[s.name] = {
                    "artifactType": {"schemaTitle": s.type, "schemaVersion": ARTIFACT_SCHEMA_VERSION}}
        outd: Dict[str, Any] = {}
        for s in comp.outputs:
            if s.kind == "parameter":
                outd.setdefault("parameters", {})[s.name] = {"type": s.type}
            else:
                outd.setdefault("artifacts", {})[s.name] = {
                    "artifactType": {"schemaTitle": s.type, "schemaVersion": ARTIFACT_SCHEMA_VERSION}}
        if ind:
            spec["inputDefinitions"] = ind
        if outd:
            spec["outputDefinitions"] = outd
        return spec


def _group_tasks(g: _Group) -> List[PipelineTask]:
    return g.all_tasks()


def _channels_of_task(t: PipelineTask) -> List[Any]:
    return [v for v in t.arguments.values() if isinstance(v, (PipelineParam, TaskOutput))]


def _channels_of_condition(c: ConditionOperator) -> List[Any]:
    return [x for x in (c.lhs, c.rhs) if isinstance(x, (PipelineParam, TaskOutput))]


def _external_channels(g: _Group) -> List[Any]:
    """Channels consumed inside group ``g`` (recursively) that are produced outside it."""
    inside = {t.name for t in g.all_tasks()}
    seen, out = set(), []

    def add(ch):
        if isinstance(ch, TaskOutput) and ch.task.name in inside:
            return
        k = _external_name(ch)
        if k not in seen:
            seen.add(k)
            out.append(ch)

    def walk(grp: _Group):
        for t in grp.tasks:
            for ch in _channels_of_task(t):
                add(ch)
        for sub in grp.groups:
            if sub.condition is not None:
                for ch in _channels_of_condition(sub.condition):
                    add(ch)
            walk(sub)
    walk(g)
    return out


def _ref_in_scope(ch, scope: _Group, is_root: bool) -> Dict[str, Any]:
    """How a task at ``scope`` refers to channel ``ch``."""
    kind, _ = _channel_type(ch)
    inside = {t.name for t in scope.tasks}
    for sub in scope.groups:
        inside.update(t.name for t in sub.all_tasks())
    if isinstance(ch, TaskOutput) and ch.task.name in inside:
        if kind == "parameter":
            return {"taskOutputParameter": {"outputParameterKey": ch.name,
                                            "producerTask": ch.task.name}}
        return {"taskOutputArtifact": {"outputArtifactKey": ch.name,
                                       "producerTask": ch.task.name}}
    if isinstance(ch, PipelineParam) and is_root:
        return {"componentInputParameter": ch.name}
    name = _external_name(ch)
    if kind == "parameter":
        return {"componentInputParameter": name}
    return {"componentInputArtifact": name}


def _producer_task_at_scope(ch, scope: _Group) -> Optional[str]:
    """Name of the task or sub-group (at ``scope`` level) that produces ``ch``."""
    if not isinstance(ch, TaskOutput):
        return None
    for t in scope.tasks:
        if t.name == ch.task.name:
            return t.name
    for sub in scope.groups:
        if any(t.name == ch.task.name for t in sub.all_tasks()):
            return sub.name
    return None


def _cond_operand(x, scope_inputs: Dict[str, str]) -> str:
    if isinstance(x, (PipelineParam, TaskOutput)):
        _, ptype = _channel_type(x)
        return f"inputs.parameters['{_external_name(x)}'].{_value_accessor(ptype)}"
    if isinstance(x, str):
        return json.dumps(x)
    if isinstance(x, bool):
        return "true" if x else "false"
    return repr(x)


def _compile_group(ctx: _Ctx, g: _Group, is_root: bool) -> Dict[str, Any]:
    tasks: Dict[str, Any] = {}
    # tasks directly in this group
    for t in g.tasks:
        comp_name = ctx.component_name(t.component)
        spec: Dict[str, Any] = {
            "taskInfo": {"name": t.display_name or t.name},
            "componentRef": {"name": comp_name},
        }
        if t.enable_caching is not None:
            spec["cachingOptions"] = {"enableCache": bool(t.enable_caching)}
        params: Dict[str, Any] = {}
        arts: Dict[str, Any] = {}
        deps = set()
        for in_spec in t.component.inputs:
            if in_spec.name not in t.arguments:
                continue
            v = t.arguments[in_spec.name]
            if isinstance(v, (PipelineParam, TaskOutput)):
                ref = _ref_in_scope(v, g, is_root)
                kind, _ = _channel_type(v)
                if in_spec.kind == "artifact" and kind != "artifact":
                    raise TypeError(f"task {t.name}: input {in_spec.name!r} expects an artifact")
                (arts if in_spec.kind == "artifact" else params)[in_spec.name] = ref
                p = _producer_task_at_scope(v, g)
                if p:
                    deps.add(p)
            else:
                if in_spec.kind == "artifact":
                    raise TypeError(f"task {t.name}: artifact input {in_spec.name!r} needs "
                                    "an upstream output or importer, got a constant")
                params[in_spec.name] = {"runtimeValue": {"constantValue":
                                                         _constant_value(v, in_spec.type)}}
        for d in t.dependent_tasks:
            owner = _producer_task_at_scope_name(d, g)
            if owner:
                deps.add(owner)
        deps.discard(t.name)
        ins: Dict[str, Any] = {}
        if params:
            ins["parameters"] = params
        if arts:
            ins["artifacts"] = arts
        if ins:
            spec["inputs"] = ins
        if deps:
            spec["dependentTasks"] = sorted(deps)
        if t.retries:
            spec["retryPolicy"] = {"maxRetryCount": t.retries}
        if t.env or t.resources:
            ext = spec.setdefault("mipipeOptions", {})
            if t.env:
                ext["env"] = dict(t.env)
            if t.resources:
                ext["resources"] = dict(t.resources)
        tasks[t.name] = spec
    # nested groups become sub-DAG components
    for sub in g.groups:
        sub_name = f"comp-{sub.name}"
        ext = _external_channels(sub)
        if sub.condition is not None:  # the gate is evaluated on the group task's own inputs
            have = {_external_name(c) for c in ext}
            for ch in _channels_of_condition(sub.condition):
                if _external_name(ch) not in have:
                    ext.append(ch)
                    have.add(_external_name(ch))
        sub_dag = _compile_group(ctx, sub, is_root=False)
        indefs: Dict[str, Any] = {}
        task_inputs: Dict[str, Any] = {}
        deps = set()
        for ch in ext:
            kind, ptype = _channel_type(ch)
            nm = _external_name(ch)
            if kind == "parameter":
                indefs.setdefault("parameters", {})[nm] = {"type": ptype}
                task_inputs.setdefault("parameters", {})[nm] = _ref_in_scope(ch, g, is_root)
            else:
                indefs.setdefault("artifacts", {})[nm] = {"artifactType": {
                    "schemaTitle": ptype, "schemaVersion": ARTIFACT_SCHEMA_VERSION}}
                task_inputs.setdefault("artifacts", {})[nm] = _ref_in_scope(ch, g, is_root)
            p = _producer_task_at_scope(ch, g)
            if p:
                deps.add(p)
        comp_spec: Dict[str, Any] = {"dag": sub_dag}
        if indefs:
            comp_spec["inputDefinitions"] = indefs
        ctx.components[sub_name] = comp_spec
        gspec: Dict[str, Any] = {"taskInfo": {"name": sub.name},
                                 "componentRef": {"name": sub_name}}
        if task_inputs:
            gspec["inputs"] = task_inputs
        if sub.condition is not None:
            c = sub.condition
            gspec["triggerPolicy"] = {"condition": f"{_cond_operand(c.lhs, {})} {c.op} "
                                                   f"{_cond_operand(c.rhs, {})}"}
        if deps:
            gspec["dependentTasks"] = sorted(deps)
        tasks[sub.name] = gspec
        if sub.exit_task is not None and sub.exit_task.name in tasks:
            et = tasks[sub.exit_task.name]
            et["triggerPolicy"] = {"strategy": "ALL_UPSTREAM_TASKS_COMPLETED"}
            et["dependentTasks"] = sorted(set(et.get("dependentTasks", [])) | {sub.name})
    return {"tasks": tasks}


def _producer_task_at_scope_name(task_name: str, scope: _Group) -> Optional[str]:
    for t in scope.tasks:
        if t.name == task_name:
            return t.name
    for sub in scope.groups:
        if any(t.name == task_name for t in sub.all_tasks()):
            return sub.name
    return None


def compile_pipeline(pipeline_func, pipeline_name: Optional[str] = None,
                     pipeline_parameters: Optional[Dict[str, Any]] = None,
                     pipeline_root: Optional[str] = None) -> Dict[str, Any]:
    if not isinstance(pipeline_func, Pipeline):
        from mipipe.dsl.pipeline import pipeline as _pl
        pipeline_func = _pl(pipeline_func)
    builder = pipeline_func.build()
    ctx = _Ctx(builder)
    root_dag = _compile_group(ctx, builder.root, is_root=True)
    root: Dict[str, Any] = {"dag": root_dag}
    params = builder.params
    if params:
        root["inputDefinitions"] = {"parameters": {p.name: {"type": p.param_type} for p in params}}
    runtime_params = {}
    overrides = dict(pipeline_parameters or {})
    for p in params:
        if p.name in overrides:
            runtime_params[p.name] = _constant_value(overrides.pop(p.name), p.param_type)
        elif p.default is not inspect.Parameter.empty and p.default is not None:
            runtime_params[p.name] = _constant_value(p.default, p.param_type)
    if overrides:
        raise ValueError(f"unknown pipeline parameters: {sorted(overrides)}")
    spec = {
        "pipelineSpec": {
            "pipelineInfo": {"name": pipeline_name or pipeline_func.name},
            "root": root,
            "components": dict(sorted(ctx.components.items())),
            "deploymentSpec": {"executors": dict(sorted(ctx.executors.items()))},
            "schemaVersion": SCHEMA_VERSION,
            "sdkVersion": SDK_VERSION,
        },
        "runtimeConfig": {"parameters": runtime_params},
    }
    if pipeline_func.description:
        spec["pipelineSpec"]["pipelineInfo"]["description"] = pipeline_func.description
    root_uri = pipeline_root or pipeline_func.pipeline_root
    if root_uri:
        spec["runtimeConfig"]["gcsOutputDirectory"] = root_uri
    return spec


class Compiler:
    """``Compiler().compile(pipeline_func, package_path)`` as in nb:231-234."""

    def compile(self, pipeline_func, package_path: str, pipeline_name: Optional[str] = None,
                pipeline_parameters: Optional[Dict[str, Any]] = None,
                type_check: bool = True) -> None:
        spec = compile_pipeline(pipeline_func, pipeline_name, pipeline_parameters)
        with open(package_path, "w") as f:
            json.dump(spec, f, indent=2, sort_keys=True)
            f.write("\n")


def component_to_yaml(comp: Component) -> str:
    """kfp-style component YAML (``output_component_file=``)."""
    import yaml
    doc = {"name": comp.name, "description": comp.description,
           "inputs": [{"name": s.name, "type": s.type} for s in comp.inputs],
           "outputs": [{"name": s.name, "type": s.type} for s in comp.outputs],
           "implementation": {"container": comp.container_spec()}}
    return yaml.safe_dump(doc, sort_keys=False)
