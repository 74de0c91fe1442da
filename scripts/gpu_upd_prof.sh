cd $GRAFT_REPO_ROOT && bash scripts/profile.sh r2upd_c --config 2 --cfk-update 1000000
