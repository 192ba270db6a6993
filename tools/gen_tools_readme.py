#!/usr/bin/env python
"""Regenerate tools/README.md: one row per script in tools/ (and tools/probe/)
from its module docstring (Python) or its leading comment block (shell, HIP).

    python tools/gen_tools_readme.py
"""
import ast
import os

HERE = os.path.dirname(os.path.abspath(__file__))
HEAD = """# tools/ — benchmarks, probes and profiling scripts

Benchmarks and probes behind the files under `profiles/`. `prof_*.sh` are `gpurun` command scripts; the one-shot
checkpoint scripts of rounds 1-5 are archived in `profiles/scripts/`; `run_steps.sh` chains GPU steps with
per-step time limits and stops at the first fault. The Python tools run on one GPU unless noted. Generated from each
file's docstring or header comment by `tools/gen_tools_readme.py`.

| File | What it does |
|---|---|
"""


def describe(path: str) -> str:
    text = open(path, encoding="utf-8", errors="replace").read()
    if path.endswith(".py"):
        try:
            doc = ast.get_docstring(ast.parse(text)) or ""
        except SyntaxError:
            doc = ""
    else:
        lines = []
        for ln in text.splitlines():
            s = ln.strip()
            if s.startswith("#!"):
                continue
            if s.startswith("#") or s.startswith("//"):
                lines.append(s.lstrip("#/ ").strip())
            elif lines or s:
                break
        doc = " ".join(x for x in lines if x)
    doc = " ".join(doc.split())
    return (doc[:217] + " ...") if len(doc) > 220 else (doc or "(no description)")


def main() -> None:
    rows = []
    for sub in ("", "probe"):
        d = os.path.join(HERE, sub)
        for name in sorted(os.listdir(d)):
            p = os.path.join(d, name)
            if os.path.isfile(p) and name.endswith((".py", ".sh", ".hip")) and name != "README.md":
                rows.append(f"| `{os.path.join(sub, name) if sub else name}` | {describe(p).replace('|', '/')} |")
    with open(os.path.join(HERE, "README.md"), "w") as f:
        f.write(HEAD + "\n".join(rows) + "\n")


if __name__ == "__main__":
    main()
