cd /root/repo; mkdir -p gpurun_out; O=gpurun_out/ab_e2e.jsonl; : > $O
for i in 1 2; do
 for v in new old; do
  if [ $v = old ]; then export KRK_LIB_PATH=kraken_amd/lib/var_oldcache/libkraken_hip.so; else unset KRK_LIB_PATH; fi
  timeout -k 10 200 python bench.py --e2e-only --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit $?
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print(json.dumps({'v':'$v','e2e':d['end_to_end']['value'],'s':d['end_to_end']['seconds']}))" >> $O
 done
done
cat $O
