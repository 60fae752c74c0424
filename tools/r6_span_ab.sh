# Round 6: obs-row layout at 65 536 envs on the final tree: pieces (default below 196 608 envs) vs
# 32-B-aligned pair spans (lid bit 0x100), interleaved.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r6k}/ab; mkdir -p $O
L=gym-usv_amd/gym_usv_amd/libusvhip.so
for r in 1 2 3; do
  O=$O LIBS=$L ROUNDS=1 bash tools/ab_libs.sh || exit $?
  O=$O LIBS=$L ROUNDS=1 VARIANT=128,263,5 bash tools/ab_libs.sh || exit $?
done
