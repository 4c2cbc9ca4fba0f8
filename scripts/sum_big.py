import csv, sys, statistics as st
d=sys.argv[1]
rows=[r for r in csv.DictReader(open(d+'/run_kernel_trace.csv'))]
obs=[int(r['End_Timestamp'])-int(r['Start_Timestamp']) for r in rows if 'k_observe' in r['Kernel_Name']]
big=[int(r['End_Timestamp'])-int(r['Start_Timestamp']) for r in rows if 'k_rollout_big' in r['Kernel_Name']]
print(d, 'obs last40 avg us %.1f' % (st.mean(obs[-40:])/1e3), 'big last20 avg us %.1f' % (st.mean(big[-20:])/1e3))
