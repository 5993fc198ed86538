import csv,collections,re,sys
D=sys.argv[1]; npass=int(sys.argv[2]); filt=sys.argv[3].split(',')
agg=collections.defaultdict(lambda: collections.defaultdict(float))
cnt=collections.defaultdict(set)
for i in range(1,npass+1):
    for r in csv.DictReader(open(f'{D}/pmc{i}/run_counter_collection.csv')):
        n=r['Kernel_Name']
        m=re.search(r'::(\w+)(<[^(]*>)?\(',n); nm=(m.group(1)+(m.group(2) or '')) if m else n[:40]
        if not any(k in nm for k in filt): continue
        key=(nm, r['Grid_Size'])
        agg[key][r['Counter_Name']]+=float(r['Counter_Value'])
        cnt[(key,r['Counter_Name'])].add(r['Dispatch_Id'])
for key,d in agg.items():
    out={c: v/len(cnt[(key,c)]) for c,v in d.items()}
    print(key, 'dispatches', len(cnt[(key,'SQ_WAVES')]))
    w=out.get('SQ_WAVE_CYCLES',1)
    print('   per-dispatch:', {c: f"{v:.4g}" for c,v in sorted(out.items())})
    print(f"   wait_any {out['SQ_WAIT_ANY']/w:.2f} wait_inst {out['SQ_WAIT_INST_ANY']/w:.2f} active {out['SQ_ACTIVE_INST_ANY']/w:.2f}  valu/mfma {out['SQ_INSTS_VALU']/max(out['SQ_INSTS_MFMA'],1):.2f}  mfma busy/(gui*4*256?) {out['SQ_VALU_MFMA_BUSY_CYCLES']/(out['GRBM_GUI_ACTIVE']/8)/1024:.3f}")
