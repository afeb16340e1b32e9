import csv, sys, re
rows=list(csv.DictReader(open(sys.argv[1])))
steps=float(sys.argv[2]) if len(sys.argv)>2 else 13
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv)>3 else 30]:
    name=re.sub(r'\(anonymous namespace\)::','',r['Name'])
    name=re.sub(r'\(.*','',name)
    print("%6.2f%% %7.1fus/step n=%4s avg=%7.1fus %s"%(100*float(r['TotalDurationNs'])/tot, float(r['TotalDurationNs'])/1e3/steps, r['Calls'], float(r['AverageNs'])/1e3, name[:90]))
print('%.3f ms/step GPU busy'%(tot/1e6/steps))
