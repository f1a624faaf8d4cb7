import os, subprocess, sys, tempfile, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import bench
bench.load_fcship()
w = tempfile.mkdtemp()
exe = os.path.join(bench.ROOT, "falcon-genome_amd", "bin", "fcs-genome")
subprocess.run([exe, "synth", "-o", w + "/d", "-c", "chr1:31000000", "-x", "30", "--no-fastq", "--noisy-frac", "0.01", "--seed", "5"], check=True, capture_output=True)
print(json.dumps(bench.bench_bgzf(w + "/d/sample.bam", 0, True)))
