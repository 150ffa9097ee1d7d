"""Fixture generator (TEST INFRASTRUCTURE ONLY; runs where /root/reference exists):
the reference's `heybuddy train` option surface and default constants as
DATA, for tests/test_cli.py's drop-in check.

Reads (as text / AST, nothing is imported or executed from the reference):
  src/python/heybuddy/__main__.py:171-244   the click decorators of `train`
  src/python/heybuddy/constants.py:73-168   the DEFAULT_* values
Writes tests/golden/cli_train_options.json:
  {"options": [{"flags": [...], "default": "<expression text>" | null,
                "flag_value": ..., "is_flag": bool}, ...],
   "constants": {"DEFAULT_...": value, ...}}

usage: python oracle/make_cli_fixture.py [/root/reference]
"""
import ast
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def constants(path):
    tree = ast.parse(open(path).read())
    env = {"int": int}
    out = {}
    for node in tree.body:
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            name = node.targets[0].id
            if not name.startswith("DEFAULT_"):
                continue
            # literals, or int(...) of earlier constants (DEFAULT_WARMUP_STEPS / DEFAULT_HOLD_STEPS)
            code = compile(ast.Expression(node.value), path, "eval")
            allowed = {n.id for n in ast.walk(node.value) if isinstance(n, ast.Name)}
            assert allowed <= set(env) | set(out), (name, allowed)
            val = eval(code, {"__builtins__": {}}, {**env, **out})
            out[name] = list(val) if isinstance(val, tuple) else val
    return out


def train_options(path):
    tree = ast.parse(open(path).read())
    fn = next(n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef) and n.name == "train")
    src = open(path).read()
    opts = []
    for dec in fn.decorator_list:
        if not (isinstance(dec, ast.Call) and getattr(dec.func, "attr", "") == "option"):
            continue
        flags = [a.value for a in dec.args if isinstance(a, ast.Constant) and str(a.value).startswith("-")]
        dest = [a.value for a in dec.args if isinstance(a, ast.Constant) and not str(a.value).startswith("-")]
        kw = {k.arg: k.value for k in dec.keywords}
        entry = {"flags": flags, "dest": dest[0] if dest else None,
                 "default": ast.get_source_segment(src, kw["default"]) if "default" in kw else None,
                 "is_flag": "is_flag" in kw or "flag_value" in kw or any("/" in f for f in flags),
                 "flag_value": ast.literal_eval(kw["flag_value"]) if "flag_value" in kw else None,
                 "multiple": "multiple" in kw}
        opts.append(entry)
    args = [a.value for d in fn.decorator_list if isinstance(d, ast.Call) and getattr(d.func, "attr", "") == "argument"
            for a in d.args[:1] if isinstance(a, ast.Constant)]
    return opts, args


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    hb = os.path.join(ref, "src", "python", "heybuddy")
    opts, args = train_options(os.path.join(hb, "__main__.py"))
    out = {"source": "reference src/python/heybuddy/__main__.py (train decorators) and constants.py, read as text",
           "arguments": args, "options": opts, "constants": constants(os.path.join(hb, "constants.py"))}
    dest = os.path.join(ROOT, "tests", "golden", "cli_train_options.json")
    with open(dest, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(opts)} options, {len(out['constants'])} constants -> {dest}")


if __name__ == "__main__":
    main()
