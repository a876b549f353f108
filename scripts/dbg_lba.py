import sys; sys.path.insert(0, '.')
from mam3slam_amd.lba import LBASolver, synthetic_problem
p = synthetic_problem(n_opt=6, n_fixed=2, n_points=120, obs_per_point=4, seed=3)
S = LBASolver()
r = S.solve(p)
print("OK", r.iterations, r.lm_trials)
