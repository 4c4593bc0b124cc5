import csv,sys,collections,glob
f=glob.glob(sys.argv[1]+"/**/*counter_collection.csv",recursive=True)[0]
agg=collections.defaultdict(lambda: collections.defaultdict(float)); disp=collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k=r["Kernel_Name"][:60]; agg[k][r["Counter_Name"]]+=float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
for k,v in agg.items():
    n=len(disp[k])
    if "gemm" in k or "wgrad" in k: print(k, n, {c: round(x/n) for c,x in v.items()})
