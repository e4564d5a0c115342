set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u scripts/ab_libs.py early=hclib_amd/lib/libhclib_amd.so noearly=hclib_amd/lib/noearly/libhclib_amd.so spectop=hclib_amd/lib/spectop/libhclib_amd.so -- sw_dag > gpurun_out/r05/ab_sw_early2.log 2>&1; tail -6 gpurun_out/r05/ab_sw_early2.log
timeout -k 10 120 python -u scripts/sw_dag_trace.py gpurun_out/r05/sw_trace.bin > gpurun_out/r05/sw_trace_early2.json 2>&1
HCLIB_AMD_LIB=hclib_amd/lib/trace_noearly/libhclib_amd.so timeout -k 10 120 python -u scripts/sw_dag_trace.py gpurun_out/r05/sw_trace.bin > gpurun_out/r05/sw_trace_noearly.json 2>&1
python3 -c "
import json
for f in ['sw_trace_early2','sw_trace_noearly']:
    d=json.load(open('gpurun_out/r05/'+f+'.json'.replace('.json','')+'.json')) if False else json.loads(open('gpurun_out/r05/'+f+'.json').read().split('\n',1)[1])
    for k in ('row','col'):
        r=d[k]; print(f,k,{kk:r[kk] for kk in ('top_from_lds','top_from_memory','left_from_memory','corner_from_memory','release_us','pickup_us','body_us','in_ingress_us','in_w0_loop_us','in_wave0_us','in_egress_us','non_sweep_per_hop_us')})
"
