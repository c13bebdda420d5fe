set -e
for rep in 1 2; do
for bb in 256 384 512 768 1280; do
  python -u scripts/multi_emulate.py --worlds 8 --delivery host-direct --rounds 3 --bounce-blocks $bb --sweep 8:4:0,8:5:0,8:10:0,8:20:0
done
done
for rep in 1 2; do
for bb in 384 768; do
  python -u scripts/multi_emulate.py --worlds 4 --delivery host-direct --rounds 3 --bounce-blocks $bb --sweep 8:2:0,8:4:0,8:5:0,8:10:0
  python -u scripts/multi_emulate.py --worlds 2 --delivery host-direct --rounds 3 --bounce-blocks $bb --sweep 8:1:0,8:2:0,8:5:0
done
done
