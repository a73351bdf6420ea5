"""Component executor: runs one lightweight component body inside a step process.

Invoked by the step container command (``python3 -m mipipe.dsl.executor_main
--component_module_path <file> --executor_input <json> --function_to_execute <fn>``),
the role ``kfp.v2.components.executor_main`` plays on Vertex Pipelines.
It maps the executor-input JSON onto the function's arguments (``InputPath`` -> local
file path of the input artifact, ``OutputPath`` -> a path to write, ``Input[T]``/
``Output[T]`` -> artifact objects, parameters -> typed values), calls the function and
writes the executor-output JSON (output parameters + artifact metadata).
"""
from __future__ import annotations

import argparse
import importlib.util
import inspect
import json
import os
import sys
from typing import Any, Dict

from mipipe.dsl import types as T
from mipipe.dsl.component import _extract_interface


def _param_from_json(v: Dict[str, Any], ptype: str, py_type=None) -> Any:
    if "intValue" in v:
        return int(v["intValue"])
    if "doubleValue" in v:
        return float(v["doubleValue"])
    if "stringValue" in v:
        s = v["stringValue"]
        if py_type is bool:
            return s.lower() in ("true", "1") if not s.startswith("{") else json.loads(s)
        if py_type in (dict, list):
            return json.loads(s)
        if py_type is int:
            return int(s)
        if py_type is float:
            return float(s)
        return s
    raise ValueError(f"unsupported parameter value {v!r}")


def _param_to_json(v: Any, ptype: str) -> Dict[str, Any]:
    if ptype == "INT":
        return {"intValue": str(int(v))}
    if ptype == "DOUBLE":
        return {"doubleValue": float(v)}
    if isinstance(v, (dict, list, bool)):
        return {"stringValue": json.dumps(v)}
    return {"stringValue": str(v)}


def _make_artifact(d: Dict[str, Any], schema: str) -> T.Artifact:
    cls = T.artifact_class_for_schema((d.get("type") or {}).get("schemaTitle", schema))
    return cls(name=d.get("name", ""), uri=d.get("uri", ""), metadata=d.get("metadata") or {})


def run_executor(func, executor_input: Dict[str, Any]) -> Dict[str, Any]:
    inputs_spec, outputs_spec = _extract_interface(func)
    ins = executor_input.get("inputs", {})
    outs = executor_input.get("outputs", {})
    in_params = ins.get("parameters", {}) or {}
    if "parameterValues" in ins:  # kfp 2.x style
        in_params = {k: _param_to_json(v, "") for k, v in ins["parameterValues"].items()}
    in_arts = ins.get("artifacts", {}) or {}
    out_arts_spec = outs.get("artifacts", {}) or {}
    out_params_spec = outs.get("parameters", {}) or {}
    kwargs: Dict[str, Any] = {}
    out_objects: Dict[str, T.Artifact] = {}
    for s in inputs_spec:
        if s.kind == "parameter":
            if s.name in in_params:
                kwargs[s.py_name] = _param_from_json(in_params[s.name], s.type, s.py_type)
            elif not s.optional:
                raise KeyError(f"missing input parameter {s.name!r}")
        else:
            lst = (in_arts.get(s.name) or {}).get("artifacts") or []
            if not lst:
                if s.optional:
                    continue
                raise KeyError(f"missing input artifact {s.name!r}")
            art = _make_artifact(lst[0], s.type)
            kwargs[s.py_name] = art.path if s.passing == "path" else art
    for s in outputs_spec:
        if s.kind != "artifact" or s.passing == "return":
            continue
        lst = (out_arts_spec.get(s.name) or {}).get("artifacts") or []
        if not lst:
            raise KeyError(f"missing output artifact spec {s.name!r}")
        art = _make_artifact(lst[0], s.type)
        os.makedirs(os.path.dirname(art.path) or ".", exist_ok=True)
        out_objects[s.name] = art
        kwargs[s.py_name] = art.path if s.passing == "path" else art

    result = func(**kwargs)

    executor_output: Dict[str, Any] = {}
    ret_specs = [s for s in outputs_spec if s.passing == "return"]
    if ret_specs:
        if len(ret_specs) == 1 and ret_specs[0].name == "Output":
            values = {"Output": result}
        else:
            values = {s.name: getattr(result, s.name) if hasattr(result, s.name) else result[i]
                      for i, s in enumerate(ret_specs)}
        params_out = {}
        for s in ret_specs:
            v = values[s.name]
            if s.kind == "parameter":
                params_out[s.name] = _param_to_json(v, s.type)
                of = (out_params_spec.get(s.name) or {}).get("outputFile")
                if of:
                    os.makedirs(os.path.dirname(of) or ".", exist_ok=True)
                    with open(of, "w") as f:
                        f.write(json.dumps(v) if isinstance(v, (dict, list, bool)) else str(v))
        if params_out:
            executor_output["parameters"] = params_out
    arts_out = {}
    for name, art in out_objects.items():
        d = art.to_dict()
        arts_out[name] = {"artifacts": [d]}
    if arts_out:
        executor_output["artifacts"] = arts_out
    return executor_output


def load_function(module_path: str, function_name: str):
    spec = importlib.util.spec_from_file_location("ephemeral_component", module_path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ephemeral_component"] = mod
    spec.loader.exec_module(mod)
    fn = getattr(mod, function_name)
    # the decorator is stripped from the shipped source; tolerate a Component too
    return getattr(fn, "python_func", fn)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="mipipe component executor")
    ap.add_argument("--component_module_path", required=True)
    ap.add_argument("--executor_input", required=True)
    ap.add_argument("--function_to_execute", required=True)
    a = ap.parse_args(argv)
    if os.environ.get("MIPIPE_GOOGLE_ALIAS", "1") == "1":
        from mipipe.storage import install_google_cloud_alias
        install_google_cloud_alias()
    ei = json.loads(a.executor_input)
    fn = load_function(a.component_module_path, a.function_to_execute)
    out = run_executor(fn, ei)
    of = ei.get("outputs", {}).get("outputFile")
    if of:
        T.write_json(of, out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
