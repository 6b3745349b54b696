for so in "$@"; do for r in 1 2; do HGA_LIB=$PWD/$so timeout -k 10 120 python bench.py --no-cpu --no-lookup --no-ingest --no-scale --steps 30 > gpurun_out/sv.json 2>/dev/null || exit 1; python3 -c "
import json,sys;d=json.load(open('gpurun_out/sv.json'));print('$so', d['ms_per_step'])"; done; done
