set -e
bash tools/dbg/r03at.sh
bash tools/dbg/r03au.sh
