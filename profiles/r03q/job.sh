# r03q: leaf size / SAH traversal cost re-swept at 128 bins, configs C and E, 2 interleaved rounds
set -e
bash tools/gpu_job.sh sweep r03q 2 "C_l4_t2=" "C_l3_t2=--leaf-size 3" "C_l5_t2=--leaf-size 5" "C_l4_t1.5=--traversal-cost 1.5" "C_l4_t2.5=--traversal-cost 2.5" \
  "E_l4_t2=--scene cornell_1m --spp 512" "E_l3_t2=--scene cornell_1m --spp 512 --leaf-size 3" "E_l5_t2=--scene cornell_1m --spp 512 --leaf-size 5" \
  "E_l4_t1.5=--scene cornell_1m --spp 512 --traversal-cost 1.5" "E_l4_t2.5=--scene cornell_1m --spp 512 --traversal-cost 2.5"
