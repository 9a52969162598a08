import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np, platform
from orc_bind import load_oracle, Template
import tunebfree_amd as T
lib = load_oracle()
t = Template(lib, seed=7)
ob, ol = t.bank()
e = T.Engine(device=-1)
tid = e.template(seed=7)
pb, pl = e.template_bank(tid)
print(platform.processor(), open('/proc/cpuinfo').read().split('model name')[1].split('\n')[0])
print('orc==prod', np.array_equal(ob.view(np.uint32), pb.view(np.uint32)), 'ndiff', int(np.sum(ob.view(np.uint32)!=pb.view(np.uint32))))
np.savez(sys.argv[1], ob=ob, pb=pb)
import math
xs = [math.sin(0.1*i+0.01) for i in range(1000)]
np.save(sys.argv[1].replace('.npz','_sin.npy'), np.array(xs))
