"""Copy a gpu_round.sh run's evidence into profiles/<round>/ and refresh profiles/pmc_traffic.json.
    python tools/summarize_round.py gpurun_out/TAG profiles/round1"""
import csv, glob, json, os, shutil, sys  # noqa: E401
from collections import defaultdict

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
tag = os.path.basename(src.rstrip('/'))
for name in ('bench', 'bench_image', 'bench_stream', 'pytest_gpu', 'smoke'):
    f = os.path.join(src, name + '.log')
    if os.path.exists(f):
        shutil.copy(f, os.path.join(dst, f'{tag}_{name}.log'))
for prof in ('prof', 'prof_image'):
    f = glob.glob(os.path.join(src, prof, '**', 'run_kernel_stats.csv'), recursive=True)
    if f:
        shutil.copy(f[0], os.path.join(dst, f'{tag}_{prof}_kernel_stats.csv'))
        print(prof)
        for r in csv.DictReader(open(f[0])):
            if 'kmp' in r['Name']:
                print(f"  {float(r['AverageNs'])/1e3:8.2f} us x{r['Calls']:>4} {r['Name'][:100]}")


def pmc(kind):
    vals = defaultdict(list)
    for ctr in ('fetch', 'write'):
        f = glob.glob(os.path.join(src, f'pmc_{ctr}{kind}', '**', 'run_counter_collection.csv'), recursive=True)
        if not f:
            return None
        shutil.copy(f[0], os.path.join(dst, f'{tag}_pmc_{ctr}{kind}.csv'))
        for r in csv.DictReader(open(f[0])):
            if 'kmp' in r['Kernel_Name']:
                # the DEC template argument: first of wave2d_u8_kernel<DEC>, second of <T, DEC, ...>
                name = r['Kernel_Name']
                if '<' not in name:  # untemplated kernels name their direction (wave2d_u8_dec_kernel)
                    direction = 'decode' if '_dec_' in name else 'encode'
                else:
                    args = [a.strip() for a in name.split('<', 1)[1].split('>', 1)[0].split(',')]
                    dec = args[0] if 'u8_kernel' in name else args[1]
                    direction = 'decode' if dec == 'true' else 'encode'
                vals[(direction, r['Counter_Name'])].append(float(r['Counter_Value']))
    out = {}
    for d in ('encode', 'decode'):
        fe = sum(vals[(d, 'FETCH_SIZE')]) / len(vals[(d, 'FETCH_SIZE')])
        wr = sum(vals[(d, 'WRITE_SIZE')]) / len(vals[(d, 'WRITE_SIZE')])
        out[d] = {'fetch_size_kb': round(fe, 1), 'write_size_kb': round(wr, 1), 'hbm_bytes': int((2 * fe + wr) * 1024)}
    out['source'] = (f'{dst}/{tag}_pmc_{{fetch,write}}{kind}.csv; rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate '
                     f'passes of bench.py --steps 3; bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950: FETCH_SIZE '
                     f'counts half of a 16-B/lane stream, MI355X_MICROARCH.md HBM)')
    return out


path = 'profiles/pmc_traffic.json'
table = json.load(open(path)) if os.path.exists(path) else {}
for kind, key in (('', 'volume_p0'), ('_image', 'image_p0')):
    t = pmc(kind)
    if t:
        table[key] = t
        print(key, json.dumps(t))
json.dump(table, open(path, 'w'), indent=1)
