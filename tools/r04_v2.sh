bash tools/round_profile.sh r04_v2 && timeout -k 10 300 python -u tools/bnin_ab.py > gpurun_out/r04_v2/bnin_ab.log 2>&1 && bash tools/r04_extra.sh
