import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
F=[r for r in rows if 'rk_burgers_wave_kernel<8' in r['Kernel_Name']]
for i,f in enumerate(F):
    s=int(f['Start_Timestamp']); e_next=int(F[i+1]['Start_Timestamp']) if i+1<len(F) else 1<<62
    it=[r for r in rows if s <= int(r['Start_Timestamp']) < e_next]
    def ms(x): return (int(x)-s)/1e6
    def span(pat):
        k=[r for r in it if pat in r['Kernel_Name']]
        if not k: return None
        return (len(k), round(ms(k[0]['Start_Timestamp']),2), round(max(ms(r['End_Timestamp']) for r in k),2), round(sum((int(r['End_Timestamp'])-int(r['Start_Timestamp'])) for r in k)/1e6,2))
    end=max(int(r['End_Timestamp']) for r in it)
    print(f'iter {i}: total {(min(e_next,end)-s)/1e6:.2f} ms  F {span("rk_burgers_wave_kernel<8")}  batch {span("nm_lane_kernel") or span("nm_fit_kernel")}  spec {span("nm_spec_kernel")}  mean {span("gp_mean_kernel")} select {span("knn_select")}')
