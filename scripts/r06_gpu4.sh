# Round 6: the N > 1 line's legs on this tree (forced at N = 1, then 2 ranks sharing the GPU), then
# the C5 back-to-back process sequence (scripts/r06_c5_seq.sh).
set -o pipefail
bash scripts/r06_legs.sh ${1:-r06g} && bash scripts/r06_c5_seq.sh ${2:-r06h}
