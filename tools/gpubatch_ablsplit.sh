# ablation: cost of splitting the A / B operands in the split-fp32 kernel (timing only; the
# ablated libraries compute wrong results)
set -o pipefail
mkdir -p gpurun_out
for L in hip ablA ablB; do
MAUV_LIB=$PWD/multimodal-auv_amd/mauv/libmauv_$L.so timeout -k 10 200 python -u tools/conv_bench.py --dtype fp32 --top 3 --trunks bathy > gpurun_out/abl_$L.log 2>&1 || exit 1
echo "$L $(grep 'TOTAL' gpurun_out/abl_$L.log | tr '\n' ' ')"
done
echo done
# build the ablated libraries first (CPU side):
#   cd multimodal-auv_amd/csrc && FL="$(make -s -p | sed -n 's/^HIPFLAGS ?= //p') -fno-slp-vectorize"
#   hipcc $FL -DABL_SPLIT_A -c conv_split.hip -o /tmp/cs_A.o   (likewise _B)
#   hipcc -shared --offload-arch=gfx950 -o ../mauv/libmauv_ablA.so $(ls build/*.o | grep -v conv_split.o) /tmp/cs_A.o
# measured (round 1c, bathy trunk shapes, G=5 B=64): all 73.0 ms -> 67.9 (A unsplit) / 68.4 (B unsplit)
