# round 3, call c: the r03b validation, then the keyver-3 AES layout A/B
bash tools/gpurun_r03b.sh || exit $?
bash tools/kv3_aes_ab.sh
