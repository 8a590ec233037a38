"""LDS instructions and bank-conflict cycles per kernel class from one rocprofv3 --pmc pass
(SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT): usage python3 scripts/pmc_lds.py <pmc dir>."""
import collections
import csv
import glob
import sys



def klass(name):
    """the kernel's own name, without namespaces and template arguments"""
    base = name.replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
    return base.rsplit("::", 1)[-1][:40]

acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for path in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(path)):
        k = klass(row["Kernel_Name"])
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
        n[(k, row["Counter_Name"])] += 1
for k, c in sorted(acc.items()):
    li, bc = c.get("SQ_INSTS_LDS", 0.0), c.get("SQ_LDS_BANK_CONFLICT", 0.0)
    if li:
        print(f"{k:40s} LDS instr {li:14.0f}  conflict cycles {bc:12.0f}  ratio {bc / li:.3f}")
