"""Instruction mix of every loop (backward branch) of one kernel in a device .s file.
usage: python tools/loopmix.py file.s kernel_substring"""
import collections
import re
import sys

L = open(sys.argv[1]).read().split("\n")
st = [i for i, l in enumerate(L) if sys.argv[2] in l and re.match(r"^[_A-Za-z]\S*:", l)]
i = st[0]
j = i
while not L[j].startswith(".Lfunc_end"):
    j += 1
body = L[i:j]
labels = {}
for k, l in enumerate(body):
    m = re.match(r"^(\.LBB\S+):", l)
    if m:
        labels[m.group(1)] = k
for k, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
    if m:
        t = m.group(1) or m.group(2)
        if t in labels and labels[t] < k:
            seg = body[labels[t]:k + 1]
            c = collections.Counter(x.strip().split(" ")[0] for x in seg
                                    if x.strip() and not x.strip().startswith((".", ";")))
            print(t, "len", len(seg), dict(c.most_common(16)))
