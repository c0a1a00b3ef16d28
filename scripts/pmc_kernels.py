import csv, glob, collections, re, sys
base=sys.argv[1]; pat=sys.argv[2]
agg=collections.defaultdict(lambda: collections.defaultdict(float)); disp=collections.defaultdict(lambda: collections.defaultdict(set))
for f in glob.glob(base+'/*/*_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        m=re.search(r'(k_\w+)', r['Kernel_Name'])
        if not m or pat not in m.group(1): continue
        k=m.group(1)
        agg[k][r['Counter_Name']]+=float(r['Counter_Value'])
        disp[k][r['Counter_Name']].add(r['Dispatch_Id'])
for k,v in sorted(agg.items()):
    n=lambda c: max(1,len(disp[k][c]))
    w=v.get('SQ_WAVES',1)
    print(k, 'launches', n('SQ_WAVES'), 'VGPR')
    print('   waves/launch %.0f  VALU/wave %.0f SALU/wave %.0f VMEM_RD/wave %.1f VMEM_WR/wave %.1f LDS/wave %.1f SMEM/wave %.1f BR/wave %.1f' % (w/n('SQ_WAVES'), v['SQ_INSTS_VALU']/w, v['SQ_INSTS_SALU']/w, v['SQ_INSTS_VMEM_RD']/w, v['SQ_INSTS_VMEM_WR']/w, v['SQ_INSTS_LDS']/w, v['SQ_INSTS_SMEM']/w, v['SQ_INSTS_BRANCH']/w))
    wc=v['SQ_WAVE_CYCLES']
    print('   wait_any %.2f wait_inst_any %.2f active_valu %.2f active_inst_any %.2f | fetch GB/launch %.3f write GB/launch %.3f | TCC hit %.3f' % (v['SQ_WAIT_ANY']/wc, v['SQ_WAIT_INST_ANY']/wc, v['SQ_ACTIVE_INST_VALU']/wc, v['SQ_ACTIVE_INST_ANY']/wc, v['FETCH_SIZE']*1024/n('FETCH_SIZE')/1e9, v['WRITE_SIZE']*1024/n('WRITE_SIZE')/1e9, v['TCC_HIT_sum']/max(1,(v['TCC_HIT_sum']+v['TCC_MISS_sum']))))
