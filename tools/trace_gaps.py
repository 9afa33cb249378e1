import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
names=[r["Kernel_Name"] for r in rows]
start=[i for i,n in enumerate(names) if "gram_kernel" in n][-3]
prev=int(rows[start]["Start_Timestamp"])
for r in rows[start:start+40]:
    s,e=int(r["Start_Timestamp"]),int(r["End_Timestamp"])
    nm=r["Kernel_Name"].split("(")[0].replace("void ","")
    print(f"{nm[:40]:40s} grid={r['Grid_Size_X']:>7}x{r['Grid_Size_Y']:>3} dur={(e-s)/1e3:7.1f}us gap={(s-prev)/1e3:6.1f}us")
    prev=e
