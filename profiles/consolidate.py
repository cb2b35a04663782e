"""Fold the one-line bench JSON files of an A/B directory into one runs.jsonl.

Every directory below profiles/ (not profiles/ itself: bench.py reads the
pmc_*.json there) that holds four or more one-line bench results (JSON
objects with a "metric" key) gets a runs.jsonl with one line per run,
{"file": <old name>, ...the bench line...}, in name order, and the files are
removed.  Paths cited in DESIGN.md / README.md and the validation runs
(final_<commit>/) stay as they are.

    python profiles/consolidate.py [--dry-run]
"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(ROOT)


def cited() -> set:
    out = set()
    for doc in ("DESIGN.md", "README.md", "INTEGRATION.md", "BASELINE.md"):
        p = os.path.join(REPO, doc)
        if os.path.exists(p):
            out |= set(re.findall(r"profiles/[A-Za-z0-9_./-]+\.json", open(p).read()))
    return out


def bench_line(path: str):
    try:
        with open(path) as f:
            text = f.read().strip()
        if "\n" in text:
            return None
        d = json.loads(text)
    except (OSError, ValueError):
        return None
    return d if isinstance(d, dict) and "metric" in d else None


def main() -> None:
    dry = "--dry-run" in sys.argv
    keep = cited()
    moved = 0
    for d, _, files in sorted(os.walk(ROOT)):
        if d == ROOT or os.path.basename(d).startswith("final_"):
            continue
        runs = []
        for name in sorted(files):
            if not name.endswith(".json"):
                continue
            rel = os.path.relpath(os.path.join(d, name), REPO)
            if rel in keep:
                continue
            b = bench_line(os.path.join(d, name))
            if b is not None:
                runs.append((name, b))
        if len(runs) < 4:
            continue
        out = os.path.join(d, "runs.jsonl")
        print(f"{os.path.relpath(d, REPO)}: {len(runs)} runs")
        moved += len(runs)
        if dry:
            continue
        with open(out, "a") as f:
            for name, b in runs:
                f.write(json.dumps({"file": name, **b}) + "\n")
        for name, _ in runs:
            os.remove(os.path.join(d, name))
    print(f"{moved} files folded")


if __name__ == "__main__":
    main()
