set -e
SKIP_TRAFFIC=1 bash tools/pmc.sh gpurun_out/pmc_v3 --spp 250
echo done
