#!/bin/bash
# round-3 batch 4/5: stitch split checks + headline / chain / tracker G sweep, then the whole suite + evidence
cd $GRAFT_REPO_ROOT
bash tools/r03_batch5.sh || exit $?
bash tools/r03_batch4.sh
