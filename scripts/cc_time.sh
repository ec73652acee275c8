cd $GRAFT_REPO_ROOT
timeout -k 5 60 ./tools/chain_check sweep | tail -1 || exit 1
for n in 4096 2048 1024 512; do timeout -k 5 30 ./tools/chain_check time $n || exit 1; done
