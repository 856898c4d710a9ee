import subprocess, sys, os
subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "patch_skdefer.py"), sys.argv[1], "21"], check=True)
