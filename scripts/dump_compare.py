import numpy as np, sys
a=np.load(sys.argv[1]); b=np.load(sys.argv[2])
print("max|phi| %.3e  max diff %.3e  rel %.3e" % (np.abs(a).max(), np.abs(a-b).max(), np.abs(a-b).max()/np.abs(a).max()))
