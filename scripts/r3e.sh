set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
BIBFS_TINY_STAMP=1 timeout -k 10 120 ./build/bin/bibfs_hip gnp:100000::6 0 99999 --resident --repeat 4 > $O/r3e_stamp.txt 2>&1 || { echo STAMP_FAILED; tail $O/r3e_stamp.txt; exit 1; }
head -9 $O/r3e_stamp.txt
timeout -k 10 60 ./build/bin/mailbox_rtt > $O/r3e_mailbox.txt 2>&1 || { echo MAILBOX_FAILED; tail $O/r3e_mailbox.txt; exit 1; }
cat $O/r3e_mailbox.txt
timeout -k 10 600 bash scripts/ab_tiny.sh > $O/r3e_ab.log 2>&1 || { echo AB_FAILED; tail $O/r3e_ab.log; exit 1; }
cat $O/ab_tiny.jsonl
