set -e
run() { timeout -k 10 200 python bench.py --path dsp --steps 200 --warmup 10 --no-cpu-baseline "$@" 2>>gpurun_out/dsp.err | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); r=d['roofline']; print('tick_us %.1f host_ms %.3f big_us %.1f GBs %.0f frac %.3f' % (r['tick']['kernel_ms']*1e3, d['p50_host_tick_ms'], r['kernel_ms']*1e3, r['achieved'], r['frac']))"; }
echo cur; run
echo cur-sorted; run --dsp-sort
echo tf64; ART_LIB=variants/libart_tf64.so run
echo tf64-sorted; ART_LIB=variants/libart_tf64.so run --dsp-sort
