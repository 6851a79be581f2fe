#!/bin/bash
# usage: tools_resusage.sh file.hip  -> one line per kernel: name VGPR AGPR spill occupancy LDS
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC ${RU_FLAGS} -c "$1" -o /tmp/_ru.o -Rpass-analysis=kernel-resource-usage 2>&1 | \
python3 -c '
import sys,re
cur=None;rows=[]
for line in sys.stdin:
    m=re.search(r"remark: +(.*?) \[-Rpass",line)
    if not m:
        if "error" in line: print(line.rstrip())
        continue
    s=m.group(1)
    if s.startswith("Function Name:"):
        cur={"name":s.split(":",1)[1].strip()};rows.append(cur)
    elif cur is not None and ":" in s:
        k,v=s.split(":",1);cur[k.strip()]=v.strip()
for r in rows:
    print(r["name"][:70].ljust(70),"V",r.get("VGPRs"),"A",r.get("AGPRs"),"Vsp",r.get("VGPRs Spill"),"Ssp",r.get("SGPRs Spill"),"occ",r.get("Occupancy [waves/SIMD]"),"lds",r.get("LDS Size [bytes/block]"))
'
