#!/usr/bin/env python3
"""Static instruction counts of the dataflow executor, per source section.

    python scripts/isa_sections.py [K G TELE DIAG WPE]   (default: 3 8 0 0 1, the config 2 launch;
                                                          WPE 4 = the build for two waves per SIMD)

Compiles csrc/dataflow.hip for gfx950 with line tables (the production flags of
build_ext.py plus -gline-tables-only), takes the instantiation
``rate_dataflow_kernel<K, G, TELE, DIAG>`` from the assembly and attributes every
instruction to the dataflow.hip line of its ``.loc`` (instructions of inlined
helpers keep their header's line; they are grouped by header).  The sections are
the numbered ``// ----`` blocks of the kernel loop, with the rating lambda split
at its DIAG clock points (priors / update / publish / records) -- the same split
``ANA_RATE_DIAG`` times.  Counts are static (each instruction once), not weighted
by how often it runs: they show which part of an iteration's dependent chain is
long, not where the time goes.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "analyzer_amd", "csrc")
SRC = os.path.join(CSRC, "dataflow.hip")


def sections():
    """(first line, name) of each section, from the source's markers."""
    out = [(1, "prologue")]
    lines = open(SRC).read().splitlines()
    for i, ln in enumerate(lines, 1):
        m = re.search(r"// -{10,} \((\d+)\) (.*)", ln)
        if m:
            out.append((i, "(%s) %s" % (m.group(1), m.group(2).strip()[:40])))
        for clock, name in (("d_p[1] = __builtin", "(10b) rating: update"),
                            ("d_p[2] = __builtin", "(10c) rating: publish"),
                            ("d_p[3] = __builtin", "(10d) rating: records")):
            if clock in ln and "d_p[0]" not in ln:
                out.append((i, name))
    return sorted(out)


def classify(op):
    if op.startswith("v_mfma"):
        return "MFMA"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("s_load", "s_buffer_load")):
        return "SMEM"
    if op.startswith("s_waitcnt"):
        return "WAIT"
    if op.startswith(("s_cbranch", "s_branch")):
        return "BR"
    if op.startswith("s_"):
        return "SALU"
    return "OTHER"


def main():
    K, G, TELE, DIAG, WPE = (sys.argv[1:6] + ["3", "8", "0", "0", "1"][len(sys.argv[1:6]):])
    diag = "true" if DIAG in ("1", "true") else "false"
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "df.s")
        cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + CSRC, "-fapprox-func",
               "-freciprocal-math", "-fno-signed-zeros", "-gline-tables-only", "--cuda-device-only",
               "-S", SRC, "-o", asm]
        subprocess.run(cmd, check=True)
        text = open(asm).read().splitlines()
    files = {}
    want = "rate_dataflow_kernelILi%sELi%sELi%sELb%dELi%sE" % (K, G, TELE, 1 if diag == "true" else 0, WPE)
    start = None
    for i, ln in enumerate(text):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
        if m:
            files[m.group(1)] = os.path.basename(m.group(3) or m.group(2))
        if start is None and ln.startswith("_ZN3ana20" + want) and ":" in ln:
            start = i
    if start is None:
        sys.exit("instantiation %s not found" % want)
    secs = sections()
    counts = collections.OrderedDict()
    cur = ("?", 0)
    vgpr = sgpr = None
    for ln in text[start + 1:]:
        s = ln.strip()
        if s.startswith(".Lfunc_end"):
            break
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            cur = (files.get(m.group(1), "?"), int(m.group(2)))
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        op = s.split()[0]
        cls = classify(op)
        f, line = cur
        if f == "dataflow.hip":
            name = [n for l0, n in secs if l0 <= line][-1] if line else "prologue"
        else:
            name = "inlined " + f
        c = counts.setdefault(name, collections.Counter())
        c[cls] += 1
    for ln in text[start:]:
        m = re.search(r"\.vgpr_count:\s+(\d+)|; NumVgprs: (\d+)", ln)
        if m and vgpr is None:
            vgpr = m.group(1) or m.group(2)
        m = re.search(r"; NumSgprs: (\d+)", ln)
        if m and sgpr is None:
            sgpr = m.group(1)
        if vgpr and sgpr:
            break
    cols = ["VALU", "SALU", "VMEM", "LDS", "SMEM", "WAIT", "BR", "MFMA", "OTHER"]
    print("rate_dataflow_kernel<%s, %s, %s, %s, %s>  (VGPRs %s, SGPRs %s), static instructions per section"
          % (K, G, TELE, diag, WPE, vgpr, sgpr))
    print("%-46s" % "section" + "".join("%7s" % c for c in cols) + "  total")
    tot = collections.Counter()
    order = [n for _, n in secs] + sorted(n for n in counts if n.startswith("inlined"))
    for name in order:
        if name not in counts:
            continue
        c = counts[name]
        tot.update(c)
        print("%-46s" % name + "".join("%7d" % c[k] for k in cols) + "  %5d" % sum(c.values()))
    for name in counts:
        if name not in order:
            c = counts[name]
            tot.update(c)
            print("%-46s" % name + "".join("%7d" % c[k] for k in cols) + "  %5d" % sum(c.values()))
    print("%-46s" % "total" + "".join("%7d" % tot[k] for k in cols) + "  %5d" % sum(tot.values()))


if __name__ == "__main__":
    main()
