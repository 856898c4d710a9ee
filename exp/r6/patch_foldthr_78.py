import subprocess, sys, os
subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "patch_foldthr.py"), sys.argv[1], "7", "8"], check=True)
