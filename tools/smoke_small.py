import sys
sys.argv=['x']
exec(open('/root/repo/tools/gpu_smoke.py').read().split("if __name__")[0])
from piadmm import config, scenario
compare('casadi_default H10', config.casadi_default(H=10), scenario.intersection(10), 40)
compare('matlab_pi H10', config.matlab_pi(H=10), scenario.intersection(10), 40)
