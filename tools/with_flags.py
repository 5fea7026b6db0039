"""Run a script with module constants overridden (A/B of fixed choices without environment switches):

    python tools/with_flags.py asrx.blocks.KEEP_IN_LN=False -- bench.py --steps 10

Each MODULE.NAME=VALUE (VALUE a Python literal) is set after importing MODULE, then the script runs as __main__."""
import ast
import importlib
import os
import runpy
import sys


def main():
    argv = sys.argv[1:]
    if "--" not in argv:
        raise SystemExit(__doc__)
    cut = argv.index("--")
    sets, rest = argv[:cut], argv[cut + 1:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "asr-transformer_amd"))
    sys.path.insert(0, root)
    for s in sets:
        lhs, val = s.split("=", 1)
        mod, name = lhs.rsplit(".", 1)
        m = importlib.import_module(mod)
        if not hasattr(m, name):
            raise SystemExit(f"{mod} has no attribute {name}")
        setattr(m, name, ast.literal_eval(val))
        print(f"[with_flags] {mod}.{name} = {getattr(m, name)!r}", file=sys.stderr)
    sys.argv = rest
    runpy.run_path(rest[0], run_name="__main__")


if __name__ == "__main__":
    main()
