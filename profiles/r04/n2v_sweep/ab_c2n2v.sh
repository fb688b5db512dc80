set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for m in sorted sweep; do
    WHARF_N2V_REWALK=$m timeout -k 10 300 python -u tools/rewalk_probe.py --model node2vec --batches 4 > gpurun_out/c2n_${m}_$rep.log 2>&1
    echo "c2 $m rep $rep: $(tail -1 gpurun_out/c2n_${m}_$rep.log | cut -c1-110)"
  done
done
