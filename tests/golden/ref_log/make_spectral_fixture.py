"""Extract the reference's own recorded spectral-clustering case from its run log
(/root/reference/src/MG_UTI_LOG_0.15, ENP75 with scaffold fraction 0.15, an older code revision):
line 333 lists the strong core connections (x, y, score) that run_clustering fed to
spectral_clustering (ReadClusteringEngine.cpp:770-772), line 335 the partition it returned.  Both
are reference *outputs*, stored as data in spectral_mg_uti.json (tests/test_clustering.py pins the
host spectral clustering against them).  Run in the container that holds the reference."""
import ast
import json
import os

LOG = "/root/reference/src/MG_UTI_LOG_0.15"
lines = open(LOG).read().splitlines()
conns = ast.literal_eval(lines[332])   # 1-based line 333
part = ast.literal_eval(lines[334])    # 1-based line 335
assert all(len(c) == 3 for c in conns) and all(isinstance(g, list) for g in part)
out = {"source": "src/MG_UTI_LOG_0.15:333 (strong core connections), :335 (spectral partition)",
       "connections": [list(c) for c in conns], "partition": part}
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "spectral_mg_uti.json"), "w") as f:
    json.dump(out, f, indent=0)
print(len(conns), "connections,", len(part), "groups")
