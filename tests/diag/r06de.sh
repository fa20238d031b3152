# Round 6: r06e (16-row tiles, C2 A/B) then r06d (tile threshold on the batch and C4, the gloo
# verify rehearsal).   (GPU box)
set -o pipefail
bash tests/diag/r06e.sh && bash tests/diag/r06d.sh
