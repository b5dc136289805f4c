for w in 1 2 4; do SA_WAVES_PER_GROUP=$w timeout -k 10 60 python tools/debug_handoff.py || exit 1; done
