# A/B of the bit-packed ReLU mask (branch exp-bitmask, files in exp/bm_overlay) against the
# tree as committed: the overlay is applied to a copy of the tree in /tmp, never in place
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$PWD
rm -rf /tmp/bmtree && mkdir /tmp/bmtree && cp -r honk_amd tests oracle bench.py __graft_entry__.py include /tmp/bmtree/
cp -r exp/bm_overlay/* /tmp/bmtree/
cd /tmp/bmtree
timeout -k 10 600 python -u -m pytest -m gpu tests/test_gpu_train_native.py tests/test_train_golden.py tests/test_gpu_cnn_train.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/bm_pytest.log 2>&1
tail -1 $R/gpurun_out/bm_pytest.log
for i in 1 2; do
  (cd $R && timeout -k 10 200 python -u bench.py --train --steps 10 --warmup 2 > gpurun_out/bm_main_$i.json 2>/dev/null)
  timeout -k 10 200 python -u bench.py --train --steps 10 --warmup 2 > $R/gpurun_out/bm_new_$i.json 2>/dev/null
  grep -o '"value": [0-9.]*' $R/gpurun_out/bm_main_$i.json $R/gpurun_out/bm_new_$i.json
done
grep -o '"parity": {[^}]*}' $R/gpurun_out/bm_new_1.json
