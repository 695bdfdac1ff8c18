"""Source rules of the native runtime that tests cannot catch by running.

The executor's and transports' device work runs on NON-blocking HIP streams,
which are not ordered after the legacy null stream. A null-stream
``hipMemset`` / ``hipMemcpy`` on memory those streams use next is therefore a
race (round 5: the fused-pass counter zeroed that way was sometimes still
garbage at the first signalling launch and the bounded frame wait timed out,
profiles/SUMMARY_r5.md section 6). Initialise such memory with the ``*Async``
form on the consuming stream (and wait for it when the host reads it)."""
import os
import re

from helpers import ROOT

RUNTIME = os.path.join(ROOT, "csrc", "runtime")


def test_no_null_stream_memset_or_memcpy_in_the_runtime():
    bad = []
    for name in sorted(os.listdir(RUNTIME)):
        if not name.endswith(".cpp"):
            continue
        src = open(os.path.join(RUNTIME, name)).read()
        src = re.sub(r"//[^\n]*", "", src)  # comments may name the rule
        for m in re.finditer(r"\bhip(Memset|Memcpy)(2D)?\s*\(", src):
            line = src.count("\n", 0, m.start()) + 1
            bad.append(f"{name}:{line}: {m.group(0)}")
    assert not bad, "null-stream memory ops in the runtime: " + ", ".join(bad)
