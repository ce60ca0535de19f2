# Round 6: whole-step A/B of the 16 x 16 patch on the K >= 4096 layers against the 8 x 16 patch everywhere.
TAG=ph16c bash scripts/gpu_r6_ab.sh "ph16k" "ph8|DG_PLAN_DISABLE=x3h16"
