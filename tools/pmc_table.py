"""Average PMC counters per kernel (first grid size seen per kernel name) from
rocprofv3 counter_collection CSVs: python tools/pmc_table.py gpurun_out/pmc*/run_counter_collection.csv"""
import csv, sys, collections
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void nr::", "")[:48] + f" g={r['Grid_Size']}"
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    if "mlp" not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.4g}")
