"""A reader for CmdStan CSV files that follows what rstan::read_stan_csv takes from
them (rstan's parse_stancsv_comments): the ``key = value`` comment lines before
"# Adaptation terminated" (leading '#', all blanks and "(Default)" stripped, split on
'='), the adaptation block (step size, diagonal inverse metric), the "Elapsed Time"
trailer, the header row and the draw rows (every line not starting with '#').
Test helper, not product code."""
from __future__ import annotations

import re

import numpy as np


def read(path):
    lines = open(path).read().splitlines()
    comments = [l for l in lines if l.startswith("#")]
    body = [l for l in lines if not l.startswith("#") and l.strip()]
    adapt = [i for i, c in enumerate(comments) if "Adaptation terminated" in c]
    end = adapt[0] if adapt else len(comments)
    values = {}
    for c in comments[:end]:
        if "=" not in c:
            continue
        c = re.sub(r"^#+\s*|\s*|\(Default\)", "", c)
        parts = c.split("=")
        values.setdefault(parts[0], parts[1] if len(parts) > 1 else "")
    stepsize, inv_metric = None, None
    if adapt:
        blk = comments[adapt[0]:]
        for j, c in enumerate(blk):
            m = re.match(r"#\s*Step size\s*=\s*(\S+)", c)
            if m:
                stepsize = float(m.group(1))
            if "Diagonal elements of inverse mass matrix" in c:
                inv_metric = np.array([float(v) for v in blk[j + 1].lstrip("#").split(",")])
    times = {}
    for c in comments:
        m = re.search(r"([0-9.]+) seconds \((Warm-up|Sampling|Total)\)", c)
        if m:
            times[m.group(2)] = float(m.group(1))
    header = body[0].split(",")
    rows = np.array([[float(v) for v in r.split(",")] for r in body[1:]]) if len(body) > 1 \
        else np.zeros((0, len(header)))
    # where the warmup rows end: CmdStan puts the adaptation block between the phases
    n_before = None
    if adapt:
        idx = lines.index(comments[adapt[0]])
        n_before = sum(1 for l in lines[:idx] if not l.startswith("#") and l.strip()) - 1
    return {"values": values, "stepsize": stepsize, "inv_metric": inv_metric, "times": times,
            "header": header, "rows": rows, "rows_before_adaptation": n_before,
            "comments": comments}
