timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/ -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b.json 2>/dev/null
python -c "import json;d=json.load(open('gpurun_out/b.json'));print(round(d['value'],1), d['bfgs_hg'], d['bfgs_hg_n4096'])"
