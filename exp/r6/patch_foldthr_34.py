import subprocess, sys, os
subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "patch_foldthr.py"), sys.argv[1], "3", "4"], check=True)
