"""Python port of the Shiny server's progress parser (ShinyInterface/server.R:457-472,
``do_progress``): it takes the last "Chain N ..." match of the sunk stdout
(stan.log), the first "(digits)%" in it and the chain number, and shows
floor(((chain - 1) * 100 + frac) / 4) percent.  Test helper, not product code."""
from __future__ import annotations

import math
import re


def do_progress(lines):
    hits = [m for line in lines for m in re.findall(r"Chain \d+.*", line)]
    if not hits:
        return None
    r = hits[-1]
    frac_s = re.search(r"(\d+)%", r)
    if frac_s is None:
        return None
    frac = float(frac_s.group(1))
    chain = int(re.search(r"Chain (\d+)", r).group(1))
    return math.floor(((chain - 1) * 100 + frac) / 4)


def replay(lines):
    """do_progress after each line, as the 1-second reactiveFileReader would see the
    file grow (server.R:474-479)."""
    return [do_progress(lines[:i + 1]) for i in range(len(lines))]
