import subprocess, sys, os
subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "patch_fold.py"), sys.argv[1], "noins"], check=True)
