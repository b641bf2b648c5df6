#!/bin/bash
# Runs D then C in one box (the pool is busy: one acquisition for both).
R=$GRAFT_REPO_ROOT
cd $R
bash profiles/r06/run_d.sh; echo "run d rc $?"
bash profiles/r06/run_c.sh; echo "run c rc $?"
