set -o pipefail
HCLIB_AMD_LIB=hclib_amd/lib/trace_noearly/libhclib_amd.so timeout -k 10 120 python -u scripts/sw_dag_trace.py gpurun_out/r05/sw_trace.bin > gpurun_out/r05/sw_trace_noearly2.json 2>&1
python3 -c "
import json
d=json.loads(open('gpurun_out/r05/sw_trace_noearly2.json').read().split('\n',1)[1])
for k in ('row','col'):
    r=d[k]; print(k,{kk:v for kk,v in r.items() if kk.endswith('_us') or kk.startswith('top')})
"
